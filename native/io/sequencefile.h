// SequenceFile v6 reader / writer in C++ (the native half of hbmr/io/sequencefile.py).
//
// Format (hadoop-1.0.3 SequenceFile.java:191-203, 915-990): "SEQ" + version 6,
// key/value class names (Text: vint length + UTF-8), compressed and
// block-compressed flags, codec class name (when compressed), metadata
// (int32 count + Text pairs), 16-byte sync hash; then records
//   int32 recordLength | int32 keyLength | key bytes | value bytes
// with a sync escape (int32 -1 + the 16-byte hash) at most every 2000 bytes,
// or, block-compressed, blocks of (escape + hash, vint nrec, and four
// codec-compressed buffers: key lengths, keys, value lengths, values).
//
// Codecs: DefaultCodec (zlib) and GzipCodec via zlib; others raise.  Split
// reading follows SequenceFileRecordReader: sync to the first marker at or
// after `start`, then read records until one begins at or after `end` right
// behind a sync marker.  Everything is big-endian on disk.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

namespace hbmr {
namespace io {

// Hadoop WritableUtils vint / vlong (bit-compatible).
void write_vlong(std::string& out, int64_t v);
int64_t read_vlong(const uint8_t*& p, const uint8_t* end);

enum class Compression { NONE, RECORD, BLOCK };

class SeqReader {
 public:
  explicit SeqReader(const std::string& path);
  ~SeqReader();
  SeqReader(const SeqReader&) = delete;
  SeqReader& operator=(const SeqReader&) = delete;

  const std::string& key_class() const { return key_class_; }
  const std::string& value_class() const { return value_class_; }
  const std::map<std::string, std::string>& metadata() const { return meta_; }
  Compression compression() const { return comp_; }
  int64_t header_end() const { return header_end_; }
  int64_t file_length() const { return file_len_; }
  const uint8_t* sync_bytes() const { return sync_; }
  const std::string& path() const { return path_; }

  int64_t position() const;
  void seek(int64_t pos);
  // Position at the first sync marker at or after pos (Reader.sync).
  void sync_to(int64_t pos);
  // Next record's serialized key/value bytes; false at end of file.
  bool next(std::string& key, std::string& value);
  // Whether the record just returned was preceded by a sync marker.
  bool sync_seen() const { return sync_seen_; }

 private:
  bool read_exact(void* dst, size_t n);
  bool read_int(int32_t& v);
  bool read_block();
  std::string decompress(const std::string& in) const;

  FILE* f_ = nullptr;
  std::string path_, key_class_, value_class_, codec_;
  std::map<std::string, std::string> meta_;
  Compression comp_ = Compression::NONE;
  uint8_t sync_[16];
  int64_t header_end_ = 0, file_len_ = 0;
  bool sync_seen_ = false;
  // block-compressed state
  std::vector<std::pair<std::string, std::string>> blk_;
  size_t blk_i_ = 0;
};

class SeqWriter {
 public:
  SeqWriter(const std::string& path, const std::string& key_class,
            const std::string& value_class,
            const std::map<std::string, std::string>& metadata = {});
  ~SeqWriter();
  void append(const std::string& key, const std::string& value);
  void close();
  int64_t length() const { return pos_; }

 private:
  void put(const void* p, size_t n);
  FILE* f_ = nullptr;
  uint8_t sync_[16];
  int64_t pos_ = 0, last_sync_ = 0;
};

// Records of a FileSplit [start, start + length) of a SequenceFile, with the
// exact boundary rule of SequenceFileRecordReader (every record belongs to
// exactly one split).
class SeqSplitReader {
 public:
  SeqSplitReader(const std::string& path, int64_t start, int64_t length);
  bool next(std::string& key, std::string& value);
  float progress() const;
  SeqReader& reader() { return r_; }

 private:
  SeqReader r_;
  int64_t start_, end_;
  bool more_;
};

// The Java FileSplit serialization (Text path, int64 start, int64 length)
// Pipes hands a C++ RecordReader (getInputSplit()).
struct FileSplitDesc {
  std::string path;
  int64_t start = 0, length = 0;
};
FileSplitDesc parse_file_split(const std::string& raw);

// FloatVectorWritable: int32 BE count + count BE float32.
void decode_float_vector(const std::string& raw, std::vector<float>& out);
std::string encode_float_vector(const float* v, int n);
int32_t decode_int_writable(const std::string& raw);
std::string encode_int_writable(int32_t v);

}  // namespace io
}  // namespace hbmr
