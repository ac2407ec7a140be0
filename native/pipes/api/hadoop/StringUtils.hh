// String helpers (API-compatible with hadoop-1.0.3/src/c++/utils/api/hadoop/StringUtils.hh).
#ifndef HBMR_STRING_UTILS_HH
#define HBMR_STRING_UTILS_HH

#include <stdint.h>

#include <string>
#include <vector>

namespace HadoopUtils {

std::string toString(int32_t x);
int32_t toInt(const std::string& val);
float toFloat(const std::string& val);
bool toBool(const std::string& val);
uint64_t getCurrentMillis();
std::vector<std::string> splitString(const std::string& str, const char* separator);
std::string quoteString(const std::string& str, const char* deliminators);
std::string unquoteString(const std::string& str);

}  // namespace HadoopUtils

#endif
