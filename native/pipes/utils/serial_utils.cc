// Pipes wire-format codecs (VInt/VLong bit-compatible with Hadoop's
// WritableUtils, cf. hadoop-1.0.3/src/c++/utils/impl/SerialUtils.cc:178-231) and
// FILE*-backed streams.
#include "hadoop/SerialUtils.hh"

#include <errno.h>
#include <string.h>

#include <cstring>
#include <sstream>

namespace HadoopUtils {

Error::Error(const std::string& msg, const std::string& file, int line,
             const std::string& function) {
  std::ostringstream o;
  o << msg << " at " << file << ":" << line << " in " << function;
  error = o.str();
}

// ---- FileInStream ------------------------------------------------------------
FileInStream::FileInStream() : mFile(NULL), isOwned(false) {}

bool FileInStream::open(const std::string& name) {
  mFile = fopen(name.c_str(), "rb");
  isOwned = true;
  return mFile != NULL;
}

bool FileInStream::open(FILE* file) {
  mFile = file;
  isOwned = false;
  return mFile != NULL;
}

void FileInStream::read(void* buf, size_t len) {
  const size_t got = fread(buf, 1, len, mFile);
  if (got != len) {
    if (feof(mFile)) throw Error("end of file");
    throw Error(std::string("read error: ") + strerror(errno));
  }
}

bool FileInStream::skip(size_t nbytes) { return fseek(mFile, (long)nbytes, SEEK_CUR) == 0; }

bool FileInStream::close() {
  int r = 0;
  if (mFile != NULL && isOwned) r = fclose(mFile);
  mFile = NULL;
  return r == 0;
}

FileInStream::~FileInStream() { close(); }

// ---- FileOutStream ---------------------------------------------------------------
FileOutStream::FileOutStream() : mFile(NULL), isOwned(false) {}

bool FileOutStream::open(const std::string& name, bool overwrite) {
  if (!overwrite) {
    FILE* f = fopen(name.c_str(), "rb");
    if (f != NULL) {
      fclose(f);
      return false;
    }
  }
  mFile = fopen(name.c_str(), "wb");
  isOwned = true;
  return mFile != NULL;
}

bool FileOutStream::open(FILE* file) {
  mFile = file;
  isOwned = false;
  return mFile != NULL;
}

void FileOutStream::write(const void* buf, size_t len) {
  if (fwrite(buf, 1, len, mFile) != len) throw Error(std::string("write error: ") + strerror(errno));
}

bool FileOutStream::advance(size_t nbytes) { return fseek(mFile, (long)nbytes, SEEK_CUR) == 0; }

void FileOutStream::flush() { fflush(mFile); }

bool FileOutStream::close() {
  int r = 0;
  if (mFile != NULL) {
    fflush(mFile);
    if (isOwned) r = fclose(mFile);
  }
  mFile = NULL;
  return r == 0;
}

FileOutStream::~FileOutStream() { close(); }

// ---- StringInStream --------------------------------------------------------------
StringInStream::StringInStream(const std::string& str) : buffer(str), itr(buffer.begin()) {}

void StringInStream::read(void* buf, size_t buflen) {
  if ((size_t)(buffer.end() - itr) < buflen) throw Error("end of string");
  std::memcpy(buf, &*itr, buflen);
  itr += (long)buflen;
}

// ---- codecs ----------------------------------------------------------------------
void serializeLong(int64_t t, OutStream& stream) {
  if (t >= -112 && t <= 127) {
    int8_t b = (int8_t)t;
    stream.write(&b, 1);
    return;
  }
  int8_t len = -112;
  if (t < 0) {
    t ^= -1ll;  // one's complement
    len = -120;
  }
  uint64_t tmp = (uint64_t)t;
  while (tmp != 0) {
    tmp >>= 8;
    --len;
  }
  stream.write(&len, 1);
  const int n = (len < -120) ? -(len + 120) : -(len + 112);
  for (int idx = n; idx != 0; --idx) {
    const int shift = (idx - 1) * 8;
    const uint8_t b = (uint8_t)(((uint64_t)t >> shift) & 0xff);
    stream.write(&b, 1);
  }
}

int64_t deserializeLong(InStream& stream) {
  int8_t first;
  stream.read(&first, 1);
  if (first >= -112) return first;
  const bool negative = first < -120;
  const int len = negative ? -(first + 120) : -(first + 112);
  uint8_t buf[8];
  stream.read(buf, (size_t)len);
  uint64_t t = 0;
  for (int i = 0; i < len; ++i) t = (t << 8) | buf[i];
  return negative ? (int64_t)(t ^ ~0ull) : (int64_t)t;
}

void serializeInt(int32_t t, OutStream& stream) { serializeLong(t, stream); }

int32_t deserializeInt(InStream& stream) { return (int32_t)deserializeLong(stream); }

void serializeFloat(float t, OutStream& stream) {
  uint32_t u;
  std::memcpy(&u, &t, 4);
  const uint8_t b[4] = {(uint8_t)(u >> 24), (uint8_t)(u >> 16), (uint8_t)(u >> 8), (uint8_t)u};
  stream.write(b, 4);
}

float deserializeFloat(InStream& stream) {
  uint8_t b[4];
  stream.read(b, 4);
  const uint32_t u = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

void deserializeFloat(float& t, InStream& stream) { t = deserializeFloat(stream); }

void serializeString(const std::string& t, OutStream& stream) {
  serializeInt((int32_t)t.size(), stream);
  if (!t.empty()) stream.write(t.data(), t.size());
}

void deserializeString(std::string& t, InStream& stream) {
  const int32_t len = deserializeInt(stream);
  HADOOP_ASSERT(len >= 0, "negative string length");
  t.resize((size_t)len);
  if (len > 0) stream.read(&t[0], (size_t)len);
}

}  // namespace HadoopUtils
