// Raw Snappy (the block format: varint length + literal/copy elements) and
// Hadoop's block framing of it, in C++ for the host side of the data path.
//
// Reference behaviour: hadoop-1.0.3 SnappyCodec.java:95-110 (BlockCompressor-
// Stream with bufferSize io.compression.codec.snappy.buffersize = 256 KiB and
// overhead bufferSize/6 + 32), BlockCompressorStream.java:76-153 (per block a
// big-endian int of the uncompressed length, then one or more big-endian
// int-length-prefixed compressed chunks of at most MAX_INPUT_SIZE input each),
// BlockDecompressorStream.java:55-110 (the reader), and the JNI wrappers
// src/native/.../snappy/Snappy{Compressor,Decompressor}.c which hand whole
// direct buffers to libsnappy.  libsnappy is not in this image, so the codec
// itself is written here from the format: a hash-table LZ77 over 64 KiB
// fragments (matches never cross a fragment, so 16-bit table entries and
// 2-byte offsets suffice), with the usual skip acceleration over
// incompressible input, and a bounds-checked decoder that accepts any valid
// stream (copies may reach back across fragments).
//
// C ABI (ctypes from hbmr/io/snappy.py, libhbmr_cpu.so).
#include <cstdint>
#include <cstring>

namespace {

constexpr int kFragment = 1 << 16;
constexpr int kHashBits = 14;

inline uint32_t load32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t load64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
inline uint32_t hash4(uint32_t v) { return (v * 0x1e35a7bdu) >> (32 - kHashBits); }

inline uint8_t* put_varint(uint8_t* o, uint32_t v) {
  while (v >= 0x80) {
    *o++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *o++ = (uint8_t)v;
  return o;
}

inline uint8_t* put_literal(uint8_t* o, const uint8_t* s, int len) {
  const uint32_t n = (uint32_t)len - 1;
  if (n < 60) {
    *o++ = (uint8_t)(n << 2);
  } else {
    int bytes = n < (1u << 8) ? 1 : n < (1u << 16) ? 2 : n < (1u << 24) ? 3 : 4;
    *o++ = (uint8_t)((59 + bytes) << 2);
    for (int i = 0; i < bytes; ++i) *o++ = (uint8_t)(n >> (8 * i));
  }
  std::memcpy(o, s, len);
  return o + len;
}

// one copy element of 4..64 bytes
inline uint8_t* put_copy_short(uint8_t* o, uint32_t off, int len) {
  if (len < 12 && off < 2048) {
    *o++ = (uint8_t)(1 | ((len - 4) << 2) | ((off >> 8) << 5));
    *o++ = (uint8_t)off;
  } else {
    *o++ = (uint8_t)(2 | ((len - 1) << 2));
    *o++ = (uint8_t)off;
    *o++ = (uint8_t)(off >> 8);
  }
  return o;
}

// a match of any length: 64-byte elements while ≥ 68 remain (so the tail is
// never shorter than 4), then one of 60 if needed, then the rest
inline uint8_t* put_copy(uint8_t* o, uint32_t off, int len) {
  while (len >= 68) {
    o = put_copy_short(o, off, 64);
    len -= 64;
  }
  if (len > 64) {
    o = put_copy_short(o, off, 60);
    len -= 60;
  }
  return put_copy_short(o, off, len);
}

// length of the common prefix of a and b, b < end
inline int match_len(const uint8_t* a, const uint8_t* b, const uint8_t* end) {
  const uint8_t* b0 = b;
  while (b + 8 <= end) {
    const uint64_t x = load64(a) ^ load64(b);
    if (x) return (int)(b - b0) + (__builtin_ctzll(x) >> 3);
    a += 8;
    b += 8;
  }
  while (b < end && *a == *b) {
    ++a;
    ++b;
  }
  return (int)(b - b0);
}

uint8_t* compress_fragment(const uint8_t* in, int n, uint8_t* o, uint16_t* table) {
  const uint8_t* lit = in;  // start of pending literal
  if (n >= 15) {
    std::memset(table, 0, sizeof(uint16_t) << kHashBits);
    const uint8_t* end = in + n;
    const uint8_t* limit = end - 4;  // last position a 4-byte load may start
    const uint8_t* p = in + 1;
    uint32_t skip = 32;
    while (p <= limit) {
      const uint32_t h = hash4(load32(p));
      const uint8_t* cand = in + table[h];
      table[h] = (uint16_t)(p - in);
      if (cand < p && load32(cand) == load32(p)) {
        if (p > lit) o = put_literal(o, lit, (int)(p - lit));
        const int len = 4 + match_len(cand + 4, p + 4, end);
        o = put_copy(o, (uint32_t)(p - cand), len);
        p += len;
        lit = p;
        skip = 32;
        // seed the table with the position just before the next search
        if (p <= limit) table[hash4(load32(p - 1))] = (uint16_t)(p - 1 - in);
        continue;
      }
      p += skip++ >> 5;
    }
  }
  if (lit < in + n) o = put_literal(o, lit, (int)(in + n - lit));
  return o;
}

inline void put_be32(uint8_t* o, uint32_t v) {
  o[0] = (uint8_t)(v >> 24);
  o[1] = (uint8_t)(v >> 16);
  o[2] = (uint8_t)(v >> 8);
  o[3] = (uint8_t)v;
}
inline uint32_t get_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// parse the varint preamble; returns bytes used or -1
int get_varint(const uint8_t* p, long n, uint32_t* v) {
  uint32_t r = 0;
  for (int i = 0; i < 5 && i < n; ++i) {
    r |= (uint32_t)(p[i] & 0x7f) << (7 * i);
    if (!(p[i] & 0x80)) {
      if (i == 4 && p[i] > 0x0f) return -1;
      *v = r;
      return i + 1;
    }
  }
  return -1;
}

}  // namespace

extern "C" {

long hbmr_snappy_max_compressed_length(long n) { return 32 + n + n / 6; }

// raw snappy of in[0:n] into out (capacity ≥ hbmr_snappy_max_compressed_length)
long hbmr_snappy_compress(const uint8_t* in, long n, uint8_t* out, long cap) {
  if (n < 0 || n > 0xffffffffL || cap < hbmr_snappy_max_compressed_length(n)) return -1;
  uint16_t table[1 << kHashBits];
  uint8_t* o = put_varint(out, (uint32_t)n);
  for (long off = 0; off < n; off += kFragment) {
    const int len = (int)(n - off < kFragment ? n - off : kFragment);
    o = compress_fragment(in + off, len, o, table);
  }
  return (long)(o - out);
}

// uncompressed length from the preamble, or -1 — also when it exceeds what
// n bytes can expand to (a 3-byte copy makes at most 64 bytes), so a corrupt
// preamble cannot make the caller allocate gigabytes
long hbmr_snappy_uncompressed_length(const uint8_t* in, long n) {
  uint32_t v;
  if (get_varint(in, n, &v) < 0 || (long)v > 22 * n + 64) return -1;
  return (long)v;
}

// decode a raw snappy stream; returns the bytes written (== the preamble's
// length) or -1 on any malformed input (truncated elements, a zero or
// out-of-range offset, output overrun, length mismatch)
long hbmr_snappy_decompress(const uint8_t* in, long n, uint8_t* out, long cap) {
  uint32_t want;
  const int h = get_varint(in, n, &want);
  if (h < 0 || (long)want > cap) return -1;
  const uint8_t* p = in + h;
  const uint8_t* end = in + n;
  uint8_t* o = out;
  uint8_t* oend = out + want;
  while (p < end) {
    const uint8_t tag = *p++;
    const int kind = tag & 3;
    if (kind == 0) {
      uint32_t len = tag >> 2;
      if (len >= 60) {
        const int bytes = (int)len - 59;
        if (end - p < bytes) return -1;
        len = 0;
        for (int i = 0; i < bytes; ++i) len |= (uint32_t)p[i] << (8 * i);
        p += bytes;
      }
      const uint64_t l = (uint64_t)len + 1;
      if ((uint64_t)(end - p) < l || (uint64_t)(oend - o) < l) return -1;
      std::memcpy(o, p, l);
      o += l;
      p += l;
      continue;
    }
    uint32_t len, off;
    if (kind == 1) {
      if (end - p < 1) return -1;
      len = 4 + ((tag >> 2) & 7);
      off = ((uint32_t)(tag >> 5) << 8) | p[0];
      p += 1;
    } else if (kind == 2) {
      if (end - p < 2) return -1;
      len = 1 + (tag >> 2);
      off = p[0] | ((uint32_t)p[1] << 8);
      p += 2;
    } else {
      if (end - p < 4) return -1;
      len = 1 + (tag >> 2);
      off = load32(p);
      p += 4;
    }
    if (off == 0 || off > (uint64_t)(o - out) || (uint64_t)(oend - o) < len) return -1;
    const uint8_t* s = o - off;
    if (off >= len) {
      std::memcpy(o, s, len);
      o += len;
    } else {
      for (uint32_t i = 0; i < len; ++i) *o++ = s[i];  // overlapping run
    }
  }
  return o == oend ? (long)want : -1;
}

// Hadoop BlockCompressorStream framing of one write(in, n) + finish(): a block
// is [int32 BE uncompressed length][int32 BE chunk length][raw snappy]… with
// each chunk compressing at most max_input = buffer_size - (buffer_size/6+32)
// bytes (SnappyCodec.java:105-109, BlockCompressorStream.java:91-137).  An
// empty input is the lone block header 0 that finish() writes.
long hbmr_snappy_hadoop_max_length(long n, int buffer_size) {
  const long max_in = buffer_size - (buffer_size / 6 + 32);
  if (max_in <= 0) return -1;
  const long chunks = n == 0 ? 0 : (n + max_in - 1) / max_in;
  return 4 + chunks * 4 + chunks * 32 + n + n / 6 + 32;
}

long hbmr_snappy_hadoop_compress(const uint8_t* in, long n, int buffer_size, uint8_t* out,
                                 long cap) {
  const long max_in = buffer_size - (buffer_size / 6 + 32);
  if (max_in <= 0 || n < 0 || n > 0x7fffffffL || cap < hbmr_snappy_hadoop_max_length(n, buffer_size))
    return -1;
  uint8_t* o = out;
  put_be32(o, (uint32_t)n);
  o += 4;
  for (long off = 0; off < n; off += max_in) {
    const long len = n - off < max_in ? n - off : max_in;
    const long c = hbmr_snappy_compress(in + off, len, o + 4, cap - (o + 4 - out));
    if (c < 0) return -1;
    put_be32(o, (uint32_t)c);
    o += 4 + c;
  }
  return (long)(o - out);
}

// total uncompressed length of a framed stream (every block's header), or -1
long hbmr_snappy_hadoop_uncompressed_length(const uint8_t* in, long n) {
  long pos = 0, total = 0;
  while (pos < n) {
    if (n - pos < 4) return -1;
    const long orig = get_be32(in + pos);
    pos += 4;
    long got = 0;
    while (got < orig) {
      if (n - pos < 4) return -1;
      const long c = get_be32(in + pos);
      pos += 4;
      if (c <= 0 || n - pos < c) return -1;
      const long u = hbmr_snappy_uncompressed_length(in + pos, c);
      if (u < 0) return -1;
      got += u;
      pos += c;
    }
    if (got != orig) return -1;
    total += orig;
  }
  return total;
}

// BlockDecompressorStream: decode every block of a framed stream into out
long hbmr_snappy_hadoop_decompress(const uint8_t* in, long n, uint8_t* out, long cap) {
  long pos = 0, w = 0;
  while (pos < n) {
    if (n - pos < 4) return -1;
    const long orig = get_be32(in + pos);
    pos += 4;
    const long start = w;
    while (w - start < orig) {
      if (n - pos < 4) return -1;
      const long c = get_be32(in + pos);
      pos += 4;
      if (c <= 0 || n - pos < c) return -1;
      const long u = hbmr_snappy_decompress(in + pos, c, out + w, cap - w);
      if (u < 0) return -1;
      w += u;
      pos += c;
    }
    if (w - start != orig) return -1;
  }
  return w;
}

}  // extern "C"
