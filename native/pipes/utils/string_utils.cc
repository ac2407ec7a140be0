// String helpers of the Pipes utilities (cf. hadoop-1.0.3/src/c++/utils/impl/StringUtils.cc).
#include "hadoop/StringUtils.hh"

#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "hadoop/SerialUtils.hh"

namespace HadoopUtils {

std::string toString(int32_t x) { return std::to_string(x); }

int32_t toInt(const std::string& val) {
  const char* begin = val.c_str();
  char* end = NULL;
  errno = 0;
  const long r = strtol(begin, &end, 10);
  HADOOP_ASSERT(errno == 0 && end != begin && *end == '\0', "problem with integer '" + val + "'");
  return (int32_t)r;
}

float toFloat(const std::string& val) {
  const char* begin = val.c_str();
  char* end = NULL;
  const float r = strtof(begin, &end);
  HADOOP_ASSERT(end != begin && *end == '\0', "problem with float '" + val + "'");
  return r;
}

bool toBool(const std::string& val) {
  if (val == "true") return true;
  if (val == "false") return false;
  HADOOP_ASSERT(false, "problem with boolean '" + val + "'");
  return false;
}

uint64_t getCurrentMillis() {
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return (uint64_t)tv.tv_sec * 1000 + (uint64_t)tv.tv_usec / 1000;
}

std::vector<std::string> splitString(const std::string& str, const char* separator) {
  std::vector<std::string> out;
  std::string::size_type start = 0;
  while (start <= str.size()) {
    const std::string::size_type next = str.find_first_of(separator, start);
    if (next == std::string::npos) {
      out.push_back(str.substr(start));
      break;
    }
    out.push_back(str.substr(start, next - start));
    start = next + 1;
  }
  return out;
}

std::string quoteString(const std::string& str, const char* deliminators) {
  std::string out;
  for (char c : str) {
    if (c == '\\' || strchr(deliminators, c) != NULL) {
      char buf[4];
      snprintf(buf, sizeof(buf), "\\%02x", (unsigned char)c);
      out += buf;
    } else {
      out += c;
    }
  }
  return out;
}

std::string unquoteString(const std::string& str) {
  std::string out;
  for (size_t i = 0; i < str.size(); ++i) {
    if (str[i] == '\\' && i + 2 < str.size()) {
      out += (char)strtol(str.substr(i + 1, 2).c_str(), NULL, 16);
      i += 2;
    } else {
      out += str[i];
    }
  }
  return out;
}

}  // namespace HadoopUtils
