// LZF codec (HDF5 filter id 32000 as registered by h5py's lzf_filter.c).
// Stream format: literal run = ctrl (L-1, <32) + L bytes; back reference = ctrl
// ((len-2)<<5 | off_hi) [+ extra len byte when len-2 >= 7] + off_lo, len in [3,264], off in [1,8192].
// Used by the h5lite reader/writer for the reference's LZF-chunked feature datasets
// (game_converter.py:55-70). Any valid LZF stream round-trips; we do not mimic liblzf's exact bytes.
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

namespace rag {

size_t lzf_decompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap) {
  size_t ip = 0, op = 0;
  while (ip < n) {
    unsigned ctrl = in[ip++];
    if (ctrl < 32) {
      size_t len = ctrl + 1;
      if (op + len > cap || ip + len > n) return 0;
      std::memcpy(out + op, in + ip, len);
      op += len;
      ip += len;
    } else {
      size_t len = ctrl >> 5;
      if (len == 7) {
        if (ip >= n) return 0;
        len += in[ip++];
      }
      if (ip >= n) return 0;
      size_t off = ((ctrl & 0x1f) << 8) + in[ip++] + 1;
      len += 2;
      if (off > op || op + len > cap) return 0;
      size_t ref = op - off;
      for (size_t k = 0; k < len; ++k) out[op + k] = out[ref + k];  // overlapping copy is intended
      op += len;
    }
  }
  return op;
}

// The hash table lives per thread and is never cleared: entries carry a per-call base offset, so
// an entry below the current call's base is stale (no 128 KB reset per 1.1 MB chunk). Matches are
// extended 8 bytes at a time (the converter's feature planes are long zero / one runs, matched at
// up to 264 bytes per back reference).
size_t lzf_compress(const uint8_t* in, size_t n, uint8_t* out, size_t cap) {
  constexpr int HLOG = 14;
  thread_local std::vector<uint64_t> htab(1u << HLOG, 0);
  thread_local uint64_t next_base = 1;
  const uint64_t base = next_base;
  next_base += n + 1;
  size_t op = 0, ip = 0, lit = 0;
  auto flush = [&](size_t upto) -> bool {
    while (lit < upto) {
      size_t run = upto - lit;
      if (run > 32) run = 32;
      if (op + 1 + run > cap) return false;
      out[op++] = (uint8_t)(run - 1);
      std::memcpy(out + op, in + lit, run);
      op += run;
      lit += run;
    }
    return true;
  };
  while (ip + 2 < n) {
    uint32_t v = ((uint32_t)in[ip] << 16) | ((uint32_t)in[ip + 1] << 8) | in[ip + 2];
    uint32_t h = (v * 2654435761u) >> (32 - HLOG);
    const uint64_t e = htab[h];
    htab[h] = base + ip;
    if (e >= base && ip - (size_t)(e - base) <= 8192) {
      const size_t ref = (size_t)(e - base);
      if (in[ref] == in[ip] && in[ref + 1] == in[ip + 1] && in[ref + 2] == in[ip + 2]) {
        size_t maxlen = n - ip;
        if (maxlen > 264) maxlen = 264;
        size_t len = 3;
        bool done = false;
        while (len + 8 <= maxlen) {
          uint64_t a, b;
          std::memcpy(&a, in + ref + len, 8);
          std::memcpy(&b, in + ip + len, 8);
          const uint64_t d = a ^ b;
          if (d) {
            len += (size_t)(__builtin_ctzll(d) >> 3);
            done = true;
            break;
          }
          len += 8;
        }
        if (!done)
          while (len < maxlen && in[ref + len] == in[ip + len]) ++len;
        if (!flush(ip)) return 0;
        size_t off = ip - ref - 1;
        size_t l2 = len - 2;
        if (l2 < 7) {
          if (op + 2 > cap) return 0;
          out[op++] = (uint8_t)((l2 << 5) | (off >> 8));
        } else {
          if (op + 3 > cap) return 0;
          out[op++] = (uint8_t)((7 << 5) | (off >> 8));
          out[op++] = (uint8_t)(l2 - 7);
        }
        out[op++] = (uint8_t)(off & 0xff);
        ip += len;
        lit = ip;
        continue;
      }
    }
    ++ip;
  }
  if (!flush(n)) return 0;
  return op;
}

}  // namespace rag
