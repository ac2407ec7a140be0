// SequenceFile v6 in C++ — see sequencefile.h.
#include "sequencefile.h"

#include <zlib.h>

#include <chrono>
#include <cstring>
#include <random>
#include <stdexcept>

namespace hbmr {
namespace io {

namespace {
constexpr int32_t kSyncEscape = -1;
constexpr int kSyncHash = 16;
constexpr int64_t kSyncInterval = 100 * (4 + kSyncHash);

inline uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
inline void put_be32(std::string& s, uint32_t v) {
  char b[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
  s.append(b, 4);
}

std::string read_text(FILE* f) {
  // vint length + bytes
  int8_t first;
  if (fread(&first, 1, 1, f) != 1) throw std::runtime_error("truncated SequenceFile header");
  uint8_t buf[9];
  buf[0] = (uint8_t)first;
  int len = 1;
  if (first < -112) {
    len = first < -120 ? -119 - first : -111 - first;
    if (fread(buf + 1, 1, len - 1, f) != (size_t)(len - 1))
      throw std::runtime_error("truncated SequenceFile header");
  }
  const uint8_t* p = buf;
  const int64_t n = read_vlong(p, buf + len);
  std::string s((size_t)n, '\0');
  if (n && fread(&s[0], 1, (size_t)n, f) != (size_t)n)
    throw std::runtime_error("truncated SequenceFile header");
  return s;
}

void put_text(std::string& out, const std::string& s) {
  write_vlong(out, (int64_t)s.size());
  out += s;
}

std::string zlib_inflate(const std::string& in, bool gzip) {
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, gzip ? 16 + MAX_WBITS : MAX_WBITS) != Z_OK)
    throw std::runtime_error("inflateInit failed");
  zs.next_in = (Bytef*)in.data();
  zs.avail_in = (uInt)in.size();
  std::string out;
  char buf[1 << 16];
  int rc;
  do {
    zs.next_out = (Bytef*)buf;
    zs.avail_out = sizeof(buf);
    rc = inflate(&zs, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) {
      inflateEnd(&zs);
      throw std::runtime_error("corrupt compressed SequenceFile data");
    }
    out.append(buf, sizeof(buf) - zs.avail_out);
  } while (rc != Z_STREAM_END);
  inflateEnd(&zs);
  return out;
}
}  // namespace

void write_vlong(std::string& out, int64_t i) {
  if (i >= -112 && i <= 127) {
    out.push_back((char)(int8_t)i);
    return;
  }
  int len = -112;
  if (i < 0) {
    i ^= -1LL;
    len = -120;
  }
  for (int64_t tmp = i; tmp != 0; tmp >>= 8) --len;
  out.push_back((char)(int8_t)len);
  len = len < -120 ? -(len + 120) : -(len + 112);
  for (int idx = len; idx != 0; --idx) {
    const int shift = (idx - 1) * 8;
    out.push_back((char)((i >> shift) & 0xFF));
  }
}

int64_t read_vlong(const uint8_t*& p, const uint8_t* end) {
  if (p >= end) throw std::runtime_error("truncated vint");
  const int8_t first = (int8_t)*p++;
  if (first >= -112) return first;
  const int len = first < -120 ? -119 - first : -111 - first;
  if (end - p < len - 1) throw std::runtime_error("truncated vint");
  int64_t i = 0;
  for (int idx = 0; idx < len - 1; ++idx) i = (i << 8) | *p++;
  const bool neg = first < -120 || (first >= -112 && first < 0);
  return neg ? (i ^ -1LL) : i;
}

// ------------------------------------------------------------------------ reader
SeqReader::SeqReader(const std::string& path) : path_(path) {
  f_ = fopen(path.c_str(), "rb");
  if (!f_) throw std::runtime_error("cannot open " + path);
  setvbuf(f_, nullptr, _IOFBF, 1 << 20);
  fseeko(f_, 0, SEEK_END);
  file_len_ = ftello(f_);
  fseeko(f_, 0, SEEK_SET);
  char magic[4];
  if (fread(magic, 1, 4, f_) != 4 || memcmp(magic, "SEQ", 3) != 0)
    throw std::runtime_error(path + " is not a SequenceFile");
  if ((uint8_t)magic[3] < 5) throw std::runtime_error("unsupported SequenceFile version");
  key_class_ = read_text(f_);
  value_class_ = read_text(f_);
  uint8_t flags[2];
  if (fread(flags, 1, 2, f_) != 2) throw std::runtime_error("truncated SequenceFile header");
  comp_ = flags[1] ? Compression::BLOCK : (flags[0] ? Compression::RECORD : Compression::NONE);
  if (comp_ != Compression::NONE) {
    codec_ = read_text(f_);
    if (codec_ != "org.apache.hadoop.io.compress.DefaultCodec" &&
        codec_ != "org.apache.hadoop.io.compress.GzipCodec")
      throw std::runtime_error("unsupported codec " + codec_);
  }
  int32_t nmeta;
  if (!read_int(nmeta)) throw std::runtime_error("truncated SequenceFile header");
  for (int i = 0; i < nmeta; ++i) {
    std::string k = read_text(f_);
    meta_[k] = read_text(f_);
  }
  if (!read_exact(sync_, kSyncHash)) throw std::runtime_error("truncated SequenceFile header");
  header_end_ = ftello(f_);
}

SeqReader::~SeqReader() {
  if (f_) fclose(f_);
}

bool SeqReader::read_exact(void* dst, size_t n) { return fread(dst, 1, n, f_) == n; }

bool SeqReader::read_int(int32_t& v) {
  uint8_t b[4];
  if (!read_exact(b, 4)) return false;
  v = (int32_t)be32(b);
  return true;
}

int64_t SeqReader::position() const { return ftello(f_); }

void SeqReader::seek(int64_t pos) {
  fseeko(f_, pos, SEEK_SET);
  blk_.clear();
  blk_i_ = 0;
}

void SeqReader::sync_to(int64_t position) {
  if (position + 4 + kSyncHash >= file_len_) {
    seek(file_len_);
    return;
  }
  if (position < header_end_) {
    seek(header_end_);
    sync_seen_ = true;
    return;
  }
  seek(position + 4);
  uint8_t win[kSyncHash];
  if (!read_exact(win, kSyncHash)) {
    seek(file_len_);
    return;
  }
  int64_t pos = position + 4;  // offset of win[0]
  int head = 0;                // ring buffer start
  for (;;) {
    bool eq = true;
    for (int i = 0; i < kSyncHash && eq; ++i) eq = win[(head + i) % kSyncHash] == sync_[i];
    if (eq) {
      seek(pos - 4);
      return;
    }
    int c = fgetc(f_);
    if (c == EOF) break;
    win[head] = (uint8_t)c;
    head = (head + 1) % kSyncHash;
    ++pos;
  }
  seek(file_len_);
}

std::string SeqReader::decompress(const std::string& in) const {
  return zlib_inflate(in, codec_ == "org.apache.hadoop.io.compress.GzipCodec");
}

bool SeqReader::read_block() {
  int32_t esc;
  if (!read_int(esc)) return false;
  if (esc != kSyncEscape) throw std::runtime_error(path_ + ": expected sync before block");
  uint8_t h[kSyncHash];
  if (!read_exact(h, kSyncHash) || memcmp(h, sync_, kSyncHash) != 0)
    throw std::runtime_error(path_ + ": sync check failure");
  sync_seen_ = true;
  // vints straight from the stream
  auto vint = [&]() -> int64_t {
    uint8_t b[9];
    if (!read_exact(b, 1)) throw std::runtime_error("truncated block");
    const int8_t first = (int8_t)b[0];
    int len = first >= -112 ? 1 : (first < -120 ? -119 - first : -111 - first);
    if (len > 1 && !read_exact(b + 1, len - 1)) throw std::runtime_error("truncated block");
    const uint8_t* p = b;
    return read_vlong(p, b + len);
  };
  const int64_t n = vint();
  std::string bufs[4];
  for (auto& b : bufs) {
    const int64_t ln = vint();
    std::string c((size_t)ln, '\0');
    if (ln && !read_exact(&c[0], (size_t)ln)) throw std::runtime_error("truncated block");
    b = decompress(c);
  }
  blk_.clear();
  blk_i_ = 0;
  const uint8_t* kl = (const uint8_t*)bufs[0].data();
  const uint8_t* kle = kl + bufs[0].size();
  const uint8_t* vl = (const uint8_t*)bufs[2].data();
  const uint8_t* vle = vl + bufs[2].size();
  size_t kp = 0, vp = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t a = read_vlong(kl, kle);
    const int64_t b = read_vlong(vl, vle);
    blk_.emplace_back(bufs[1].substr(kp, (size_t)a), bufs[3].substr(vp, (size_t)b));
    kp += (size_t)a;
    vp += (size_t)b;
  }
  return true;
}

bool SeqReader::next(std::string& key, std::string& value) {
  sync_seen_ = false;
  if (comp_ == Compression::BLOCK) {
    if (blk_i_ >= blk_.size() && !read_block()) return false;
    key.swap(blk_[blk_i_].first);
    value.swap(blk_[blk_i_].second);
    ++blk_i_;
    return true;
  }
  int32_t len;
  if (!read_int(len)) return false;
  if (len == kSyncEscape) {
    uint8_t h[kSyncHash];
    if (!read_exact(h, kSyncHash) || memcmp(h, sync_, kSyncHash) != 0)
      throw std::runtime_error(path_ + ": sync check failure");
    sync_seen_ = true;
    if (!read_int(len)) return false;
  }
  int32_t klen;
  if (!read_int(klen) || klen < 0 || klen > len) throw std::runtime_error("corrupt record");
  key.resize((size_t)klen);
  value.resize((size_t)(len - klen));
  if ((klen && !read_exact(&key[0], (size_t)klen)) ||
      (len - klen && !read_exact(&value[0], (size_t)(len - klen))))
    throw std::runtime_error("truncated record");
  if (comp_ == Compression::RECORD) value = decompress(value);
  return true;
}

// ------------------------------------------------------------------------ writer
SeqWriter::SeqWriter(const std::string& path, const std::string& key_class,
                     const std::string& value_class,
                     const std::map<std::string, std::string>& metadata) {
  f_ = fopen(path.c_str(), "wb");
  if (!f_) throw std::runtime_error("cannot create " + path);
  std::mt19937_64 rng((uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^
                      (uint64_t)(uintptr_t)this);
  for (int i = 0; i < kSyncHash; i += 8) {
    const uint64_t r = rng();
    memcpy(sync_ + i, &r, 8);
  }
  std::string h("SEQ\x06", 4);
  put_text(h, key_class);
  put_text(h, value_class);
  h.push_back(0);  // not compressed
  h.push_back(0);  // not block-compressed
  put_be32(h, (uint32_t)metadata.size());
  for (const auto& kv : metadata) {
    put_text(h, kv.first);
    put_text(h, kv.second);
  }
  h.append((const char*)sync_, kSyncHash);
  put(h.data(), h.size());
}

SeqWriter::~SeqWriter() { close(); }

void SeqWriter::put(const void* p, size_t n) {
  if (fwrite(p, 1, n, f_) != n) throw std::runtime_error("write failed");
  pos_ += (int64_t)n;
}

void SeqWriter::append(const std::string& key, const std::string& value) {
  if (pos_ >= last_sync_ + kSyncInterval && last_sync_ != pos_) {
    std::string s;
    put_be32(s, (uint32_t)kSyncEscape);
    s.append((const char*)sync_, kSyncHash);
    put(s.data(), s.size());
    last_sync_ = pos_;
  }
  std::string r;
  put_be32(r, (uint32_t)(key.size() + value.size()));
  put_be32(r, (uint32_t)key.size());
  put(r.data(), r.size());
  put(key.data(), key.size());
  put(value.data(), value.size());
}

void SeqWriter::close() {
  if (f_) {
    fclose(f_);
    f_ = nullptr;
  }
}

// ------------------------------------------------------------------------ splits
SeqSplitReader::SeqSplitReader(const std::string& path, int64_t start, int64_t length)
    : r_(path), start_(start), end_(start + length) {
  if (start_ > r_.position()) r_.sync_to(start_);
  start_ = r_.position();
  more_ = start_ < end_;
}

bool SeqSplitReader::next(std::string& key, std::string& value) {
  if (!more_) return false;
  const int64_t pos = r_.position();
  if (!r_.next(key, value) || (pos >= end_ && r_.sync_seen())) {
    more_ = false;
    return false;
  }
  return true;
}

float SeqSplitReader::progress() const {
  if (end_ == start_) return 0.f;
  const float p = (float)(r_.position() - start_) / (float)(end_ - start_);
  return p < 1.f ? p : 1.f;
}

FileSplitDesc parse_file_split(const std::string& raw) {
  const uint8_t* p = (const uint8_t*)raw.data();
  const uint8_t* e = p + raw.size();
  FileSplitDesc d;
  const int64_t n = read_vlong(p, e);
  if (e - p < n + 16) throw std::runtime_error("bad FileSplit");
  d.path.assign((const char*)p, (size_t)n);
  p += n;
  auto be64 = [](const uint8_t* q) {
    return (int64_t)((uint64_t)be32(q) << 32 | be32(q + 4));
  };
  d.start = be64(p);
  d.length = be64(p + 8);
  if (d.path.rfind("file:", 0) == 0) d.path = d.path.substr(5);
  return d;
}

void decode_float_vector(const std::string& raw, std::vector<float>& out) {
  if (raw.size() < 4) throw std::runtime_error("bad FloatVectorWritable");
  const uint8_t* p = (const uint8_t*)raw.data();
  const int32_t n = (int32_t)be32(p);
  if (n < 0 || raw.size() < 4 + 4 * (size_t)n) throw std::runtime_error("bad FloatVectorWritable");
  out.resize((size_t)n);
  for (int32_t i = 0; i < n; ++i) {
    const uint32_t u = be32(p + 4 + 4 * i);
    memcpy(&out[i], &u, 4);
  }
}

std::string encode_float_vector(const float* v, int n) {
  std::string s;
  s.reserve(4 + 4 * (size_t)n);
  put_be32(s, (uint32_t)n);
  for (int i = 0; i < n; ++i) {
    uint32_t u;
    memcpy(&u, &v[i], 4);
    put_be32(s, u);
  }
  return s;
}

int32_t decode_int_writable(const std::string& raw) {
  if (raw.size() < 4) throw std::runtime_error("bad IntWritable");
  return (int32_t)be32((const uint8_t*)raw.data());
}

std::string encode_int_writable(int32_t v) {
  std::string s;
  put_be32(s, (uint32_t)v);
  return s;
}

}  // namespace io
}  // namespace hbmr
