#pragma once
#include <algorithm>
#include <string>

namespace hbmr {
std::string sha1(const std::string& msg);
std::string hmacSha1(const std::string& key, const std::string& msg);
std::string base64(const std::string& in);
// base64(HMAC-SHA1(password, msg)) — the Pipes authentication digest
std::string createDigest(const std::string& password, const std::string& msg);
}  // namespace hbmr
