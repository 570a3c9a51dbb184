// json.cc — parser / serializer for jsk::Json (RFC 8259 subset: no comments;
// \uXXXX escapes incl. surrogate pairs are decoded to UTF-8).
#include "json.h"

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace jsk {

namespace {

struct Parser {
    const std::string& s;
    size_t i = 0;
    explicit Parser(const std::string& t) : s(t) {}

    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i));
    }
    void ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool lit(const char* w) {
        size_t n = std::strlen(w);
        if (s.compare(i, n, w) == 0) { i += n; return true; }
        return false;
    }
    static void utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) out += (char)cp;
        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
        } else {
            out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
            out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
        }
    }
    uint32_t hex4() {
        if (i + 4 > s.size()) fail("short \\u escape");
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            char c = s[i++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else fail("bad \\u escape");
        }
        return v;
    }
    std::string str() {
        if (s[i] != '"') fail("expected string");
        ++i;
        std::string out;
        while (true) {
            if (i >= s.size()) fail("unterminated string");
            char c = s[i++];
            if (c == '"') break;
            if (c != '\\') { out += c; continue; }
            if (i >= s.size()) fail("bad escape");
            char e = s[i++];
            switch (e) {
                case '"': out += '"'; break;
                case '\\': out += '\\'; break;
                case '/': out += '/'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'n': out += '\n'; break;
                case 'r': out += '\r'; break;
                case 't': out += '\t'; break;
                case 'u': {
                    uint32_t cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
                        i += 2;
                        uint32_t lo = hex4();
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8(out, cp);
                    break;
                }
                default: fail("bad escape");
            }
        }
        return out;
    }
    Json value() {
        ws();
        if (i >= s.size()) fail("unexpected end");
        char c = s[i];
        if (c == '{') {
            ++i;
            Json o = Json::object();
            ws();
            if (i < s.size() && s[i] == '}') { ++i; return o; }
            while (true) {
                ws();
                std::string k = str();
                ws();
                if (i >= s.size() || s[i] != ':') fail("expected ':'");
                ++i;
                o[k] = value();
                ws();
                if (i < s.size() && s[i] == ',') { ++i; continue; }
                if (i < s.size() && s[i] == '}') { ++i; return o; }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            ++i;
            Json a = Json::array();
            ws();
            if (i < s.size() && s[i] == ']') { ++i; return a; }
            while (true) {
                a.push_back(value());
                ws();
                if (i < s.size() && s[i] == ',') { ++i; continue; }
                if (i < s.size() && s[i] == ']') { ++i; return a; }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') return Json(str());
        if (lit("true")) return Json(true);
        if (lit("false")) return Json(false);
        if (lit("null")) return Json();
        size_t st = i;
        bool integral = true;
        if (s[i] == '-') ++i;
        while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
        if (i < s.size() && (s[i] == '.' || s[i] == 'e' || s[i] == 'E')) {
            integral = false;
            ++i;
            while (i < s.size() && (std::isdigit((unsigned char)s[i]) || s[i] == '-' || s[i] == '+' || s[i] == 'e' ||
                                    s[i] == 'E'))
                ++i;
        }
        if (i == st) fail("unexpected character");
        std::string num = s.substr(st, i - st);
        if (integral) return Json((int64_t)std::stoll(num));
        return Json(std::stod(num));
    }
};

void dump_str(std::string& out, const std::string& v) {
    out += '"';
    for (unsigned char c : v) {
        switch (c) {
            case '"': out += "\\\""; break;
            case '\\': out += "\\\\"; break;
            case '\n': out += "\\n"; break;
            case '\r': out += "\\r"; break;
            case '\t': out += "\\t"; break;
            default:
                if (c < 0x20) {
                    char b[8];
                    std::snprintf(b, sizeof b, "\\u%04x", c);
                    out += b;
                } else {
                    out += (char)c;
                }
        }
    }
    out += '"';
}

void dump_to(std::string& out, const Json& j) {
    switch (j.type()) {
        case Json::Null: out += "null"; break;
        case Json::Bool: out += j.as_bool() ? "true" : "false"; break;
        case Json::Int: out += std::to_string(j.as_int()); break;
        case Json::Double: {
            char b[40];
            std::snprintf(b, sizeof b, "%.17g", j.as_double());
            out += b;
            break;
        }
        case Json::String: dump_str(out, j.as_string()); break;
        case Json::Array: {
            out += '[';
            bool first = true;
            for (const auto& e : j.elems()) {
                if (!first) out += ',';
                first = false;
                dump_to(out, e);
            }
            out += ']';
            break;
        }
        case Json::Object: {
            out += '{';
            bool first = true;
            for (const auto& kv : j.items()) {
                if (!first) out += ',';
                first = false;
                dump_str(out, kv.first);
                out += ':';
                dump_to(out, kv.second);
            }
            out += '}';
            break;
        }
    }
}

}  // namespace

Json Json::parse(const std::string& text) {
    Parser p(text);
    Json v = p.value();
    p.ws();
    if (p.i != text.size()) p.fail("trailing characters");
    return v;
}

std::string Json::dump() const {
    std::string out;
    dump_to(out, *this);
    return out;
}

bool Json::operator==(const Json& o) const {
    if (t_ != o.t_) return false;
    switch (t_) {
        case Null: return true;
        case Bool: return b_ == o.b_;
        case Int: return i_ == o.i_;
        case Double: return d_ == o.d_;
        case String: return s_ == o.s_;
        case Array: return a_ == o.a_;
        case Object: return o_ == o.o_;
    }
    return false;
}

}  // namespace jsk
