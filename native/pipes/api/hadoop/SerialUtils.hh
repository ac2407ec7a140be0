// Serialization utilities of the Pipes wire format (API-compatible with
// hadoop-1.0.3/src/c++/utils/api/hadoop/SerialUtils.hh).
//   serializeInt/Long : Hadoop VInt/VLong (WritableUtils-compatible)
//   serializeFloat    : 4-byte big-endian IEEE-754 (XDR)
//   serializeString   : VInt length + bytes
#ifndef HBMR_SERIAL_UTILS_HH
#define HBMR_SERIAL_UTILS_HH

#include <stdint.h>
#include <stdio.h>

#include <string>

namespace HadoopUtils {

class Error {
 public:
  explicit Error(const std::string& msg) : error(msg) {}
  Error(const std::string& msg, const std::string& file, int line, const std::string& function);
  const std::string& getMessage() const { return error; }

 private:
  std::string error;
};

#define HADOOP_ASSERT(CONDITION, MESSAGE)                                           \
  do {                                                                              \
    if (!(CONDITION)) {                                                             \
      throw HadoopUtils::Error((MESSAGE), __FILE__, __LINE__, __func__);            \
    }                                                                               \
  } while (0)

class InStream {
 public:
  virtual void read(void* buf, size_t len) = 0;
  virtual ~InStream() {}
};

class OutStream {
 public:
  virtual void write(const void* buf, size_t len) = 0;
  virtual void flush() = 0;
  virtual ~OutStream() {}
};

class FileInStream : public InStream {
 public:
  FileInStream();
  bool open(const std::string& name);
  bool open(FILE* file);
  void read(void* buf, size_t buflen) override;
  bool skip(size_t nbytes);
  bool close();
  ~FileInStream() override;

 private:
  FILE* mFile;
  bool isOwned;
};

class FileOutStream : public OutStream {
 public:
  FileOutStream();
  bool open(const std::string& name, bool overwrite);
  bool open(FILE* file);
  void write(const void* buf, size_t len) override;
  bool advance(size_t nbytes);
  void flush() override;
  bool close();
  ~FileOutStream() override;

 private:
  FILE* mFile;
  bool isOwned;
};

class StringInStream : public InStream {
 public:
  explicit StringInStream(const std::string& str);
  void read(void* buf, size_t buflen) override;

 private:
  const std::string& buffer;
  std::string::const_iterator itr;
};

class StringOutStream : public OutStream {
 public:
  void write(const void* buf, size_t len) override { buffer.append((const char*)buf, len); }
  void flush() override {}
  std::string buffer;
};

void serializeInt(int32_t t, OutStream& stream);
int32_t deserializeInt(InStream& stream);
void serializeLong(int64_t t, OutStream& stream);
int64_t deserializeLong(InStream& stream);
void serializeFloat(float t, OutStream& stream);
float deserializeFloat(InStream& stream);
void deserializeFloat(float& t, InStream& stream);
void serializeString(const std::string& t, OutStream& stream);
void deserializeString(std::string& t, InStream& stream);

}  // namespace HadoopUtils

#endif
