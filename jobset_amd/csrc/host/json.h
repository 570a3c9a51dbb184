// json.h — minimal JSON value for the host-side mirror of the reference's
// webhook / controller objects (Kubernetes objects travel as JSON, as they do
// in an AdmissionReview). Objects keep keys sorted (std::map); numbers are
// int64 when integral, else double.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace jsk {

class Json {
public:
    enum Type { Null, Bool, Int, Double, String, Array, Object };

    Json() : t_(Null) {}
    Json(std::nullptr_t) : t_(Null) {}
    Json(bool b) : t_(Bool), b_(b) {}
    Json(int v) : t_(Int), i_(v) {}
    Json(int64_t v) : t_(Int), i_(v) {}
    Json(uint32_t v) : t_(Int), i_(v) {}
    Json(double v) : t_(Double), d_(v) {}
    Json(const char* s) : t_(String), s_(s) {}
    Json(std::string s) : t_(String), s_(std::move(s)) {}

    static Json array() { Json j; j.t_ = Array; return j; }
    static Json object() { Json j; j.t_ = Object; return j; }

    Type type() const { return t_; }
    bool is_null() const { return t_ == Null; }
    bool is_object() const { return t_ == Object; }
    bool is_array() const { return t_ == Array; }
    bool is_string() const { return t_ == String; }
    bool is_number() const { return t_ == Int || t_ == Double; }

    bool as_bool() const { return t_ == Bool ? b_ : false; }
    int64_t as_int() const { return t_ == Int ? i_ : t_ == Double ? (int64_t)d_ : 0; }
    double as_double() const { return t_ == Double ? d_ : t_ == Int ? (double)i_ : 0.0; }
    const std::string& as_string() const {
        static const std::string empty;
        return t_ == String ? s_ : empty;
    }

    // object access
    bool has(const std::string& k) const { return t_ == Object && o_.count(k) > 0; }
    const Json& get(const std::string& k) const {
        static const Json null;
        if (t_ != Object) return null;
        auto it = o_.find(k);
        return it == o_.end() ? null : it->second;
    }
    Json& operator[](const std::string& k) {  // creates the object / member
        if (t_ != Object) { *this = object(); }
        return o_[k];
    }
    void erase(const std::string& k) { if (t_ == Object) o_.erase(k); }
    const std::map<std::string, Json>& items() const { return o_; }
    std::map<std::string, Json>& items() { return o_; }

    // array access
    size_t size() const { return t_ == Array ? a_.size() : t_ == Object ? o_.size() : 0; }
    const Json& at(size_t i) const { return a_.at(i); }
    Json& at(size_t i) { return a_.at(i); }
    void push_back(Json v) {
        if (t_ != Array) *this = array();
        a_.push_back(std::move(v));
    }
    const std::vector<Json>& elems() const { return a_; }
    std::vector<Json>& elems() { return a_; }

    std::string dump() const;
    static Json parse(const std::string& text);  // throws std::runtime_error

    bool operator==(const Json& o) const;
    bool operator!=(const Json& o) const { return !(*this == o); }

private:
    Type t_;
    bool b_ = false;
    int64_t i_ = 0;
    double d_ = 0;
    std::string s_;
    std::vector<Json> a_;
    std::map<std::string, Json> o_;
};

// String-map helpers for metadata.labels / annotations / spec.nodeSelector.
// A missing map reads as empty; `has_key` distinguishes "" from absent, like
// Go's `v, ok := m[k]`.
inline bool has_key(const Json& m, const std::string& k) { return m.is_object() && m.has(k); }
inline std::string str_at(const Json& m, const std::string& k) { return m.get(k).as_string(); }

}  // namespace jsk
