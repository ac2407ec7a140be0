// HMAC-SHA1 + base64 for the Pipes job-token handshake.
//
// The reference links OpenSSL for this (src/c++/pipes/impl/HadoopPipes.cc:395-446:
// HMAC_Init/EVP_sha1 then BIO base64).  hbmr implements the two primitives
// directly (FIPS 180-1 SHA-1, RFC 2104 HMAC, RFC 4648 base64) so the task
// binaries have no OpenSSL ABI dependency.
#include "hmac_sha1.h"

#include <cstdint>
#include <cstring>

namespace hbmr {
namespace {

inline uint32_t rol(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

struct Sha1 {
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  unsigned char block[64];
  size_t used = 0;
  uint64_t total = 0;

  void compress(const unsigned char* p) {
    uint32_t w[80];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 |
             (uint32_t)p[4 * i + 2] << 8 | (uint32_t)p[4 * i + 3];
    for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; ++i) {
      uint32_t f, k;
      if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
      else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
      else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
      else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
      const uint32_t t = rol(a, 5) + f + e + k + w[i];
      e = d; d = c; c = rol(b, 30); b = a; a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
  }

  void update(const void* data, size_t n) {
    const unsigned char* p = static_cast<const unsigned char*>(data);
    total += n;
    while (n) {
      const size_t take = std::min(n, (size_t)64 - used);
      std::memcpy(block + used, p, take);
      used += take; p += take; n -= take;
      if (used == 64) { compress(block); used = 0; }
    }
  }

  void final(unsigned char out[20]) {
    const uint64_t bits = total * 8;
    const unsigned char pad = 0x80;
    update(&pad, 1);
    const unsigned char zero = 0;
    while (used != 56) update(&zero, 1);
    unsigned char len[8];
    for (int i = 0; i < 8; ++i) len[i] = (unsigned char)(bits >> (56 - 8 * i));
    update(len, 8);
    for (int i = 0; i < 5; ++i) {
      out[4 * i] = (unsigned char)(h[i] >> 24);
      out[4 * i + 1] = (unsigned char)(h[i] >> 16);
      out[4 * i + 2] = (unsigned char)(h[i] >> 8);
      out[4 * i + 3] = (unsigned char)h[i];
    }
  }
};

}  // namespace

std::string sha1(const std::string& msg) {
  Sha1 s;
  s.update(msg.data(), msg.size());
  unsigned char d[20];
  s.final(d);
  return std::string(reinterpret_cast<char*>(d), 20);
}

std::string hmacSha1(const std::string& key, const std::string& msg) {
  std::string k = key.size() > 64 ? sha1(key) : key;
  k.resize(64, '\0');
  std::string ipad(64, '\0'), opad(64, '\0');
  for (int i = 0; i < 64; ++i) {
    ipad[i] = (char)(k[i] ^ 0x36);
    opad[i] = (char)(k[i] ^ 0x5c);
  }
  return sha1(opad + sha1(ipad + msg));
}

std::string base64(const std::string& in) {
  static const char* tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    const uint32_t v = (uint8_t)in[i] << 16 | (uint8_t)in[i + 1] << 8 | (uint8_t)in[i + 2];
    out += tbl[v >> 18]; out += tbl[(v >> 12) & 63]; out += tbl[(v >> 6) & 63]; out += tbl[v & 63];
  }
  if (i < in.size()) {
    uint32_t v = (uint8_t)in[i] << 16;
    if (i + 1 < in.size()) v |= (uint8_t)in[i + 1] << 8;
    out += tbl[v >> 18];
    out += tbl[(v >> 12) & 63];
    out += (i + 1 < in.size()) ? tbl[(v >> 6) & 63] : '=';
    out += '=';
  }
  return out;
}

std::string createDigest(const std::string& password, const std::string& msg) {
  return base64(hmacSha1(password, msg));
}

}  // namespace hbmr
