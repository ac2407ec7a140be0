// Map-output buffer kernels for CPU tasks: batch partition, sort, group and
// IFile encode of serialised (key, value) records.
//
// The reference's MapOutputBuffer (hadoop-1.0.3/src/mapred/org/apache/hadoop/
// mapred/MapTask.java:869-1465) keeps records in a byte buffer with a 16-byte
// accounting entry each, quick-sorts the entries by (partition, raw key)
// (compare 1119-1130, QuickSort) and writes IFile segments per partition
// (IFile.java:119-188).  hbmr's Python collector appends the serialised bytes
// and hands whole spills to these routines, so the per-record work left in
// Python is the user's map() and the key/value serialisation.
//
// Key kinds (raw comparators / hashCode of org.apache.hadoop.io types):
//   0 TEXT   VInt length + bytes; compare bytes unsigned then length
//            (Text.Comparator); hash WritableComparator.hashBytes (31*h+b, h0=1,
//            signed bytes) over the payload
//   1 BYTES  4-byte BE length + bytes (BytesWritable); same compare / hash
//   2 INT    4-byte BE signed (IntWritable); hash = value
//   3 LONG   8-byte BE signed (LongWritable); hash = (int)(v ^ v>>>32)
//   4 RAW    whole serialised key, memcmp then length; hash = hashBytes(all)
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

namespace {

enum Kind { TEXT = 0, BYTES = 1, INT = 2, LONG = 3, RAW = 4 };

inline int vint_size(int8_t first) {
  if (first >= -112) return 1;
  if (first < -120) return -119 - first;
  return -111 - first;
}

// payload [p, p+n) of a serialised key of this kind
inline void payload(int kind, const uint8_t* k, int64_t len, const uint8_t** p, int64_t* n) {
  switch (kind) {
    case TEXT: {
      int s = vint_size(static_cast<int8_t>(k[0]));
      *p = k + s;
      *n = len - s;
      return;
    }
    case BYTES:
      *p = k + 4;
      *n = len - 4;
      return;
    default:
      *p = k;
      *n = len;
  }
}

inline int32_t be32(const uint8_t* p) {
  return static_cast<int32_t>((uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) |
                              (uint32_t(p[2]) << 8) | uint32_t(p[3]));
}

inline int64_t be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return static_cast<int64_t>(v);
}

inline int32_t hash_bytes(const uint8_t* p, int64_t n) {
  uint32_t h = 1;
  for (int64_t i = 0; i < n; ++i) h = 31u * h + static_cast<uint32_t>(static_cast<int8_t>(p[i]));
  return static_cast<int32_t>(h);
}

inline int32_t java_hash(int kind, const uint8_t* k, int64_t len) {
  if (kind == INT) return be32(k);
  if (kind == LONG) {
    uint64_t v = static_cast<uint64_t>(be64(k));
    return static_cast<int32_t>(static_cast<uint32_t>(v ^ (v >> 32)));
  }
  const uint8_t* p;
  int64_t n;
  payload(kind, k, len, &p, &n);
  return hash_bytes(p, n);
}

inline int compare(int kind, const uint8_t* a, int64_t la, const uint8_t* b, int64_t lb) {
  if (kind == INT) {
    int32_t x = be32(a), y = be32(b);
    return (x > y) - (x < y);
  }
  if (kind == LONG) {
    int64_t x = be64(a), y = be64(b);
    return (x > y) - (x < y);
  }
  const uint8_t *pa, *pb;
  int64_t na, nb;
  payload(kind, a, la, &pa, &na);
  payload(kind, b, lb, &pb, &nb);
  int c = std::memcmp(pa, pb, static_cast<size_t>(std::min(na, nb)));
  if (c) return c;
  return (na > nb) - (na < nb);
}

inline int put_vint(uint8_t* out, int64_t v) {
  // WritableUtils.writeVLong
  if (v >= -112 && v <= 127) {
    out[0] = static_cast<uint8_t>(static_cast<int8_t>(v));
    return 1;
  }
  int len = -112;
  if (v < 0) {
    v ^= -1LL;
    len = -120;
  }
  int64_t tmp = v;
  while (tmp != 0) {
    tmp >>= 8;
    --len;
  }
  out[0] = static_cast<uint8_t>(static_cast<int8_t>(len));
  int n = (len < -120) ? -(len + 120) : -(len + 112);
  for (int idx = n; idx != 0; --idx) {
    int shift = (idx - 1) * 8;
    out[1 + n - idx] = static_cast<uint8_t>((v >> shift) & 0xFF);
  }
  return 1 + n;
}

}  // namespace

extern "C" {

// part[i] = (hashCode(key_i) & INT_MAX) % R  (HashPartitioner.java:31-34)
void hbmr_hash_partition(int kind, const uint8_t* kbuf, const int64_t* kpos,
                         const int64_t* klen, int64_t n, int R, int32_t* part) {
  for (int64_t i = 0; i < n; ++i) {
    int32_t h = java_hash(kind, kbuf + kpos[i], klen[i]);
    part[i] = static_cast<int32_t>((h & 0x7fffffff) % R);
  }
}

// perm = stable order of records by (part, key)
void hbmr_sort_records(int kind, const uint8_t* kbuf, const int64_t* kpos, const int64_t* klen,
                       int64_t n, const int32_t* part, int64_t* perm) {
  std::iota(perm, perm + n, int64_t(0));
  // counting pass by partition first (R is small), then a comparison sort per
  // partition range: fewer comparisons than one sort on the pair
  int32_t R = 0;
  for (int64_t i = 0; i < n; ++i) R = std::max(R, part[i] + 1);
  std::vector<int64_t> start(static_cast<size_t>(R) + 1, 0);
  for (int64_t i = 0; i < n; ++i) ++start[part[i] + 1];
  for (int32_t r = 0; r < R; ++r) start[r + 1] += start[r];
  std::vector<int64_t> pos(start.begin(), start.end() - 1);
  for (int64_t i = 0; i < n; ++i) perm[pos[part[i]]++] = i;
  for (int32_t r = 0; r < R; ++r) {
    int64_t* lo = perm + start[r];
    int64_t* hi = perm + start[r + 1];
    if (kind == INT || kind == LONG) {
      std::stable_sort(lo, hi, [&](int64_t a, int64_t b) {
        return compare(kind, kbuf + kpos[a], 0, kbuf + kpos[b], 0) < 0;
      });
    } else {
      std::stable_sort(lo, hi, [&](int64_t a, int64_t b) {
        return compare(kind, kbuf + kpos[a], klen[a], kbuf + kpos[b], klen[b]) < 0;
      });
    }
  }
}

// ends of runs of equal keys within perm[lo, hi): writes run end positions
// (exclusive, absolute into perm) and returns the number of runs
int64_t hbmr_group_runs(int kind, const uint8_t* kbuf, const int64_t* kpos, const int64_t* klen,
                        const int64_t* perm, int64_t lo, int64_t hi, int64_t* ends) {
  int64_t nr = 0;
  for (int64_t i = lo + 1; i <= hi; ++i) {
    if (i == hi) {
      ends[nr++] = i;
      break;
    }
    int64_t a = perm[i - 1], b = perm[i];
    if (compare(kind, kbuf + kpos[a], klen[a], kbuf + kpos[b], klen[b]) != 0)
      ends[nr++] = i;
  }
  return nr;
}

// IFile segment body for records perm[lo, hi): VInt klen, VInt vlen, key,
// value ...; then the EOF marker (-1, -1).  ``out`` must hold
// sum(klen + vlen) + 10 * (hi - lo) + 2 bytes.  Returns bytes written.
// Records are (kpos, klen) / (vpos, vlen) slices of kbuf / vbuf.
int64_t hbmr_ifile_encode(const uint8_t* kbuf, const int64_t* kpos, const int64_t* klen,
                          const uint8_t* vbuf, const int64_t* vpos, const int64_t* vlen,
                          const int64_t* perm, int64_t lo, int64_t hi, uint8_t* out) {
  uint8_t* o = out;
  for (int64_t i = lo; i < hi; ++i) {
    int64_t r = perm[i];
    int64_t kl = klen[r], vl = vlen[r];
    o += put_vint(o, kl);
    o += put_vint(o, vl);
    std::memcpy(o, kbuf + kpos[r], static_cast<size_t>(kl));
    o += kl;
    std::memcpy(o, vbuf + vpos[r], static_cast<size_t>(vl));
    o += vl;
  }
  o += put_vint(o, -1);
  o += put_vint(o, -1);
  return o - out;
}

// Decode an IFile body into key/value offset arrays (for merges and reduces).
// Returns the number of records, or -1 if the buffer is malformed / capacity
// ``cap`` too small.  kpos/vpos are start offsets into ``buf``, klen/vlen sizes.
int64_t hbmr_ifile_decode(const uint8_t* buf, int64_t n, int64_t cap, int64_t* kpos,
                          int64_t* klen, int64_t* vpos, int64_t* vlen) {
  int64_t pos = 0, nr = 0;
  auto get = [&](int64_t* v) -> bool {
    if (pos >= n) return false;
    int8_t first = static_cast<int8_t>(buf[pos]);
    int sz = vint_size(first);
    if (pos + sz > n) return false;
    if (sz == 1) {
      *v = first;
    } else {
      int64_t x = 0;
      for (int i = 1; i < sz; ++i) x = (x << 8) | buf[pos + i];
      *v = (first < -120 || (first >= -112 && first < 0)) ? (x ^ -1LL) : x;
    }
    pos += sz;
    return true;
  };
  while (pos < n) {
    int64_t kl, vl;
    if (!get(&kl) || !get(&vl)) return -1;
    if (kl == -1 && vl == -1) return nr;
    if (kl < 0 || vl < 0 || pos + kl + vl > n || nr >= cap) return -1;
    kpos[nr] = pos;
    klen[nr] = kl;
    vpos[nr] = pos + kl;
    vlen[nr] = vl;
    pos += kl + vl;
    ++nr;
  }
  return nr;
}

}  // extern "C"
