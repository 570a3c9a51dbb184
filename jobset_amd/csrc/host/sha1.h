// sha1.h — SHA-1 (FIPS 180-4) for the JobSet job key: the reference labels
// every child Job and pod with hex(sha1("<ns>/<jobName>"))
// (jobHashKey / sha1Hash, pkg/controllers/jobset_controller.go:809-818).
#pragma once
#include <cstdint>
#include <string>

namespace jsk {

std::string sha1_hex(const std::string& msg);

}  // namespace jsk
