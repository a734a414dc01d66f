// Wire codec for ciphertext vectors (host code): the byte format of
// Paillier.serialize / Paillier.ciphertext_from (paillier.py:244-271) —
// pickle of an np.ndarray(dtype=object) of RawCiphertext(value, exp) — to and
// from flat little-endian word buffers, without creating a Python object per
// element.
//
// Encoder: protocol-4 opcodes, unframed, numpy's ndarray reduce
// (numpy.core.multiarray._reconstruct, loadable by numpy 1.x and 2.x),
// RawCiphertext as NEWOBJ + BUILD({'value': int, 'exp': int}) with the class
// and the two keys memoised once; values as LONG1/LONG4.
// Decoder: a small pickle machine for the opcodes CPython emits for that
// object graph at protocols 2-5 (framing, memo forms, GLOBAL/STACK_GLOBAL),
// including the reference's gmpy2 values (REDUCE of gmpy2.from_binary on
// gmpy2's binary format: type 0x01, sign byte, little-endian magnitude).
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace xhe {
namespace wire {

// f(0..T-1) on T threads (the calling thread runs part 0)
template <class F>
void run_parallel(int T, F&& f) {
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(f, t);
  f(0);
  for (auto& x : th) x.join();
}

struct Writer {
  uint8_t* out;
  int64_t cap, n = 0;
  void put(uint8_t b) {
    if (n < cap) out[n] = b;
    ++n;
  }
  void put(const void* p, int64_t len) {
    if (n + len <= cap) memcpy(out + n, p, (size_t)len);
    n += len;
  }
  void u32(uint32_t v) {
    for (int i = 0; i < 4; ++i) put((uint8_t)(v >> (8 * i)));
  }
  void str(const char* s) {  // SHORT_BINUNICODE
    size_t len = strlen(s);
    put(0x8c);
    put((uint8_t)len);
    put(s, (int64_t)len);
  }
  void binint(int32_t v) {
    if (v >= 0 && v < 256) {
      put('K');
      put((uint8_t)v);
    } else {
      put('J');
      u32((uint32_t)v);
    }
  }
  void binint64(int64_t v) {  // shape entries
    if (v >= 0 && v < 256) {
      put('K');
      put((uint8_t)v);
    } else if (v >= INT32_MIN && v <= INT32_MAX) {
      put('J');
      u32((uint32_t)v);
    } else {
      uint8_t b[9];
      int len = 0;
      for (; len < 8; ++len) b[len] = (uint8_t)((uint64_t)v >> (8 * len));
      put(0x8a);
      put((uint8_t)len);
      put(b, len);
    }
  }
};

// non-negative little-endian words -> LONG1/LONG4 (minimal two's complement)
inline void put_long(Writer& w, const uint32_t* words, int nw) {
  int top = nw - 1;
  while (top >= 0 && words[top] == 0) --top;
  int64_t bits = 0;
  if (top >= 0) bits = 32 * top + (32 - __builtin_clz(words[top]));
  int64_t nbytes = bits == 0 ? 0 : (bits + 8) / 8;  // one sign bit of room
  if (nbytes < 256) {
    w.put(0x8a);
    w.put((uint8_t)nbytes);
  } else {
    w.put(0x8b);
    w.u32((uint32_t)nbytes);
  }
  // little-endian words are the little-endian bytes; at most one zero byte
  // of sign room lies beyond the top word
  int64_t have = std::min<int64_t>(nbytes, 4 * (int64_t)nw);
  w.put(words, have);
  for (int64_t i = have; i < nbytes; ++i) w.put((uint8_t)0);
}

inline void emit_header_a(Writer& w) {
  w.put(0x80);
  w.put(4);
  w.str("numpy.core.multiarray");
  w.str("_reconstruct");
  w.put(0x93);
  w.str("numpy");
  w.put(0x94);  // memo 0: 'numpy'
  w.str("ndarray");
  w.put(0x93);
  w.put('K');
  w.put(0);
  w.put(0x85);
  w.put('C');
  w.put(1);
  w.put('b');
  w.put(0x87);
  w.put('R');
  w.put('(');  // state tuple
  w.put('K');
  w.put(1);
  w.put('(');
}

inline void emit_header_b(Writer& w) {
  w.put('t');
  w.put('h');
  w.put(0);  // 'numpy'
  w.str("dtype");
  w.put(0x93);
  w.str("O8");
  w.put(0x89);
  w.put(0x88);
  w.put(0x87);
  w.put('R');
  w.put('(');
  w.put('K');
  w.put(3);
  w.str("|");
  w.put('N');
  w.put('N');
  w.put('N');
  w.binint(-1);
  w.binint(-1);
  w.put('K');
  w.put(63);
  w.put('t');
  w.put('b');     // dtype state
  w.put(0x89);    // is_fortran = False
  w.put(']');
}

inline void emit_header(Writer& w, const int64_t* shape, int ndim) {
  emit_header_a(w);
  for (int d = 0; d < ndim; ++d) w.binint64(shape[d]);  // the shape tuple's entries
  emit_header_b(w);
}

// element i of count: RawCiphertext as NEWOBJ + BUILD({'value': v, 'exp': e});
// APPENDS batches of 1000 (what CPython emits for a list)
inline void emit_elem(Writer& w, const uint32_t* row, int n2w, int32_t e, int64_t i, int64_t count) {
  if (i % 1000 == 0) w.put('(');
  if (i == 0) {
    w.str("common.crypto.paillier.paillier");
    w.str("RawCiphertext");
    w.put(0x93);
    w.put(0x94);  // memo 1: the class
  } else {
    w.put('h');
    w.put(1);
  }
  w.put(')');
  w.put(0x81);  // NEWOBJ
  w.put('}');
  w.put('(');
  if (i == 0) {
    w.str("value");
    w.put(0x94);  // memo 2
  } else {
    w.put('h');
    w.put(2);
  }
  put_long(w, row, n2w);
  if (i == 0) {
    w.str("exp");
    w.put(0x94);  // memo 3
  } else {
    w.put('h');
    w.put(3);
  }
  w.binint(e);
  w.put('u');
  w.put('b');
  if (i % 1000 == 999 || i == count - 1) w.put('e');
}

inline void emit_footer(Writer& w) {
  w.put('t');  // state tuple
  w.put('b');  // ndarray.__setstate__
  w.put('.');
}

// Bytes of LONG1/LONG4 payload for a non-negative value (put_long's rule:
// minimal two's complement, one sign bit of room).
inline int64_t long_nbytes(const uint32_t* row, int nw) {
  int top = nw - 1;
  while (top >= 0 && row[top] == 0) --top;
  if (top < 0) return 0;
  const int64_t bits = 32 * (int64_t)top + (32 - __builtin_clz(row[top]));
  return (bits + 8) / 8;
}

// Size of element i's bytes, as emit_elem writes them (i > 0: closed form).
inline int64_t elem_bytes(const uint32_t* row, int n2w, int32_t e, int64_t i, int64_t count) {
  if (i == 0) {
    Writer w{nullptr, 0};
    emit_elem(w, row, n2w, e, 0, count);
    return w.n;
  }
  const int64_t nb = long_nbytes(row, n2w);
  int64_t s = 8 + (nb < 256 ? 2 : 5) + nb + 2 + ((e >= 0 && e < 256) ? 2 : 5) + 2;
  if (i % 1000 == 0) s += 1;
  if (i % 1000 == 999 || i == count - 1) s += 1;
  return s;
}

// emit_elem for i > 0 with direct stores (the hot loop of serialize).
inline uint8_t* write_elem(uint8_t* d, const uint32_t* row, int n2w, int32_t e, int64_t i, int64_t count) {
  static const uint8_t pre[8] = {'h', 1, ')', 0x81, '}', '(', 'h', 2};
  if (i % 1000 == 0) *d++ = '(';
  memcpy(d, pre, 8);
  d += 8;
  const int64_t nb = long_nbytes(row, n2w);
  if (nb < 256) {
    *d++ = 0x8a;
    *d++ = (uint8_t)nb;
  } else {
    *d++ = 0x8b;
    for (int k = 0; k < 4; ++k) *d++ = (uint8_t)((uint64_t)nb >> (8 * k));
  }
  const int64_t have = std::min<int64_t>(nb, 4 * (int64_t)n2w);
  memcpy(d, row, (size_t)have);
  d += have;
  for (int64_t k = have; k < nb; ++k) *d++ = 0;
  *d++ = 'h';
  *d++ = 3;
  if (e >= 0 && e < 256) {
    *d++ = 'K';
    *d++ = (uint8_t)e;
  } else {
    *d++ = 'J';
    for (int k = 0; k < 4; ++k) *d++ = (uint8_t)((uint32_t)e >> (8 * k));
  }
  *d++ = 'u';
  *d++ = 'b';
  if (i % 1000 == 999 || i == count - 1) *d++ = 'e';
  return d;
}

// Returns the byte count; writes only when out != nullptr and it fits in cap.
// Elements are sized, prefix-summed and written by `threads` host threads
// over contiguous element ranges (the bytes do not depend on the split).
inline int64_t encode(const uint32_t* ct, const int32_t* exps, int64_t count, int n2w, const int64_t* shape, int ndim,
                      uint8_t* out, int64_t cap, int threads = 1) {
  Writer hw{nullptr, 0};
  emit_header(hw, shape, ndim);
  const int64_t head = hw.n;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, count / 4096));
  std::vector<int64_t> part(T + 1, 0);  // element range bounds
  for (int t = 0; t <= T; ++t) part[t] = count * t / T;
  std::vector<int64_t> bytes(T, 0);
  run_parallel(T, [&](int t) {
    int64_t b = 0;
    for (int64_t i = part[t]; i < part[t + 1]; ++i) b += elem_bytes(ct + (size_t)i * n2w, n2w, exps[i], i, count);
    bytes[t] = b;
  });
  std::vector<int64_t> off(T + 1, head);
  for (int t = 0; t < T; ++t) off[t + 1] = off[t] + bytes[t];
  const int64_t total = off[T] + 3;
  if (!out || total > cap) return total;
  Writer h{out, cap};
  emit_header(h, shape, ndim);
  run_parallel(T, [&](int t) {
    uint8_t* d = out + off[t];
    int64_t i = part[t];
    if (i == 0 && i < part[t + 1]) {  // the first element memoises the class and keys
      Writer w{d, bytes[t]};
      emit_elem(w, ct, n2w, exps[0], 0, count);
      d += w.n;
      ++i;
    }
    for (; i < part[t + 1]; ++i) d = write_elem(d, ct + (size_t)i * n2w, n2w, exps[i], i, count);
  });
  Writer f{out + off[T], 3};
  emit_footer(f);
  return total;
}

// Where the bytes of `encode` go: straight (pos -> out + pos) or as the
// content of one zstd frame of raw blocks of `blk` bytes (14-byte frame
// header, 3-byte block headers; pos -> its block's payload).
struct Sink {
  uint8_t* out;
  int64_t blk;  // 0: unframed
  void copy(int64_t pos, const uint8_t* src, int64_t len) const {
    if (!blk) {
      memcpy(out + pos, src, (size_t)len);
      return;
    }
    while (len > 0) {
      const int64_t b = pos / blk, in = pos - b * blk, n = std::min(len, blk - in);
      memcpy(out + 14 + b * (blk + 3) + 3 + in, src, (size_t)n);
      pos += n;
      src += n;
      len -= n;
    }
  }
};

// `encode` written through a Sink: every thread encodes its element range
// into a small local buffer (cache-resident) and copies it to the Sink's
// positions, so a framed payload is written once, not as a pickle and then
// again as the frame (the intermediate pickle cost its own page faults and a
// ~30 ms munmap per 1 M ciphertexts on the GPU box). Returns the pickle's
// byte count; writes nothing when out == nullptr (size query).
inline int64_t encode_to(const uint32_t* ct, const int32_t* exps, int64_t count, int n2w, const int64_t* shape,
                         int ndim, const Sink* sink, int threads = 1) {
  Writer hw{nullptr, 0};
  emit_header(hw, shape, ndim);
  const int64_t head = hw.n;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, count / 4096));
  std::vector<int64_t> part(T + 1, 0);
  for (int t = 0; t <= T; ++t) part[t] = count * t / T;
  std::vector<int64_t> bytes(T, 0);
  run_parallel(T, [&](int t) {
    int64_t b = 0;
    for (int64_t i = part[t]; i < part[t + 1]; ++i) b += elem_bytes(ct + (size_t)i * n2w, n2w, exps[i], i, count);
    bytes[t] = b;
  });
  std::vector<int64_t> off(T + 1, head);
  for (int t = 0; t < T; ++t) off[t + 1] = off[t] + bytes[t];
  const int64_t total = off[T] + 3;
  if (!sink) return total;
  {
    std::vector<uint8_t> hb((size_t)head);
    Writer h{hb.data(), head};
    emit_header(h, shape, ndim);
    sink->copy(0, hb.data(), head);
  }
  run_parallel(T, [&](int t) {
    constexpr int64_t kBuf = 64 << 10;
    std::vector<uint8_t> loc((size_t)kBuf + 8192);  // + one element's bytes of headroom
    int64_t pos = off[t], fill = 0;
    int64_t i = part[t];
    if (i == 0 && i < part[t + 1]) {
      Writer w{loc.data(), (int64_t)loc.size()};
      emit_elem(w, ct, n2w, exps[0], 0, count);
      fill = w.n;
      ++i;
    }
    for (; i < part[t + 1]; ++i) {
      fill = write_elem(loc.data() + fill, ct + (size_t)i * n2w, n2w, exps[i], i, count) - loc.data();
      if (fill >= kBuf) {
        sink->copy(pos, loc.data(), fill);
        pos += fill;
        fill = 0;
      }
    }
    if (fill) sink->copy(pos, loc.data(), fill);
  });
  uint8_t foot[3];
  Writer f{foot, 3};
  emit_footer(f);
  sink->copy(off[T], foot, 3);
  return total;
}

// ---- the same bytes in two steps, for rows that arrive in pieces (the
// serialize pipeline: bit lengths first, then the words chunk by chunk).
// An element's size depends on its value only through the bit length.
inline int64_t elem_bytes_bits(int bits, int n2w, int32_t e, int64_t i, int64_t count) {
  if (i == 0) {  // a row of that bit length: the same LONG size as the value
    std::vector<uint32_t> row((size_t)n2w, 0u);
    if (bits > 0) row[(size_t)(bits - 1) / 32] = 1u << ((bits - 1) % 32);
    return elem_bytes(row.data(), n2w, e, 0, count);
  }
  const int64_t nb = bits == 0 ? 0 : (bits + 8) / 8;
  int64_t s = 8 + (nb < 256 ? 2 : 5) + nb + 2 + ((e >= 0 && e < 256) ? 2 : 5) + 2;
  if (i % 1000 == 0) s += 1;
  if (i % 1000 == 999 || i == count - 1) s += 1;
  return s;
}

// Pickle offsets off[0..count] of every element (off[count]: the footer)
// from the bit lengths; returns the pickle's byte count. With a sink, also
// writes the header and the footer (rows go through write_rows).
inline int64_t layout(const int16_t* bits, const int32_t* exps, int64_t count, int n2w, const int64_t* shape,
                      int ndim, int64_t* off, const Sink* sink, int threads = 1) {
  Writer hw{nullptr, 0};
  emit_header(hw, shape, ndim);
  const int64_t head = hw.n;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, count / 4096));
  std::vector<int64_t> part(T + 1, 0), tot(T + 1, 0);
  for (int t = 0; t <= T; ++t) part[t] = count * t / T;
  run_parallel(T, [&](int t) {  // per-part sizes into off[] (exclusive prefix inside the part)
    int64_t b = 0;
    for (int64_t i = part[t]; i < part[t + 1]; ++i) {
      off[i] = b;
      b += elem_bytes_bits(bits[i], n2w, exps[i], i, count);
    }
    tot[t + 1] = b;
  });
  tot[0] = head;
  for (int t = 0; t < T; ++t) tot[t + 1] += tot[t];
  run_parallel(T, [&](int t) {
    for (int64_t i = part[t]; i < part[t + 1]; ++i) off[i] += tot[t];
  });
  off[count] = tot[T];
  const int64_t total = tot[T] + 3;
  if (sink) {
    std::vector<uint8_t> hb((size_t)head);
    Writer h{hb.data(), head};
    emit_header(h, shape, ndim);
    sink->copy(0, hb.data(), head);
    uint8_t foot[3];
    Writer f{foot, 3};
    emit_footer(f);
    sink->copy(tot[T], foot, 3);
  }
  return total;
}

// ---- the same layout element range by element range, for words whose bit
// lengths arrive chunk by chunk too (an encryption still running when the
// serialize starts): the header's size first (off[0]), then each range's
// offsets from the offset its first element starts at, the footer last.
inline int64_t head_bytes(const int64_t* shape, int ndim) {
  Writer hw{nullptr, 0};
  emit_header(hw, shape, ndim);
  return hw.n;
}
inline void write_head(const int64_t* shape, int ndim, const Sink& sink) {
  const int64_t head = head_bytes(shape, ndim);
  std::vector<uint8_t> hb((size_t)head);
  Writer h{hb.data(), head};
  emit_header(h, shape, ndim);
  sink.copy(0, hb.data(), head);
}
// off[lo + 1 .. hi] from off[lo] and the bit lengths of elements lo .. hi-1
// (bits[0] = element lo's)
inline void layout_part(const int16_t* bits, const int32_t* exps, int64_t lo, int64_t hi, int64_t count, int n2w,
                        int64_t* off) {
  for (int64_t i = lo; i < hi; ++i) off[i + 1] = off[i] + elem_bytes_bits(bits[i - lo], n2w, exps[i], i, count);
}
// the same from the rows themselves (rows[0] = element lo): the bit lengths
// are read off each row's top word (the words are on the host anyway when the
// rows are written next; no device pass that would queue behind running kernels)
inline void layout_part_rows(const uint32_t* rows, const int32_t* exps, int64_t lo, int64_t hi, int64_t count,
                             int n2w, int64_t* off, int threads = 1) {
  const int64_t n = hi - lo;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n / 4096));
  std::vector<int64_t> tot((size_t)T + 1, 0);
  run_parallel(T, [&](int t) {  // per element: its size into off[i + 1], exclusive prefix within the part
    const int64_t a = lo + n * t / T, b = lo + n * (t + 1) / T;
    int64_t acc = 0;
    for (int64_t i = a; i < b; ++i) {
      const uint32_t* r = rows + (size_t)(i - lo) * n2w;
      int k = n2w - 1;
      while (k >= 0 && r[k] == 0u) --k;
      const int bits = k < 0 ? 0 : 32 * k + 32 - __builtin_clz(r[k]);
      acc += elem_bytes_bits(bits, n2w, exps[i], i, count);
      off[i + 1] = acc;
    }
    tot[(size_t)t + 1] = acc;
  });
  tot[0] = off[lo];
  for (int t = 0; t < T; ++t) tot[(size_t)t + 1] += tot[(size_t)t];
  run_parallel(T, [&](int t) {
    const int64_t a = lo + n * t / T, b = lo + n * (t + 1) / T;
    for (int64_t i = a; i < b; ++i) off[i + 1] += tot[(size_t)t];
  });
}
inline void write_foot(int64_t at, const Sink& sink) {
  uint8_t foot[3];
  Writer f{foot, 3};
  emit_footer(f);
  sink.copy(at, foot, 3);
}

// Elements lo .. hi-1 (rows: their words, row lo first) at the offsets of
// `layout`. Returns false when a row's size disagrees with its offsets (its
// bit length was not the one the layout was made from).
inline bool write_rows(const uint32_t* rows, const int32_t* exps, int64_t lo, int64_t hi, int64_t count, int n2w,
                       const int64_t* off, const Sink& sink, int threads = 1) {
  const int64_t n = hi - lo;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n / 2048));
  std::vector<char> ok((size_t)T, 1);
  run_parallel(T, [&](int t) {
    constexpr int64_t kBuf = 64 << 10;
    std::vector<uint8_t> loc((size_t)kBuf + 8192);
    const int64_t a = lo + n * t / T, b = lo + n * (t + 1) / T;
    int64_t pos = off[a], fill = 0;
    for (int64_t i = a; i < b; ++i) {
      const uint32_t* row = rows + (size_t)(i - lo) * n2w;
      int64_t len;
      if (i == 0) {
        Writer w{loc.data() + fill, (int64_t)loc.size() - fill};
        emit_elem(w, row, n2w, exps[0], 0, count);
        len = w.n;
      } else {
        len = write_elem(loc.data() + fill, row, n2w, exps[i], i, count) - (loc.data() + fill);
      }
      if (len != off[i + 1] - off[i]) {
        ok[t] = 0;
        return;
      }
      fill += len;
      if (fill >= kBuf) {
        sink.copy(pos, loc.data(), fill);
        pos += fill;
        fill = 0;
      }
    }
    if (fill) sink.copy(pos, loc.data(), fill);
  });
  for (char c : ok)
    if (!c) return false;
  return true;
}

// The same bytes written one put() at a time (the specification the fast
// encoder is checked against in tests/native/host_fuzz.cpp).
inline int64_t encode_reference(const uint32_t* ct, const int32_t* exps, int64_t count, int n2w, const int64_t* shape,
                                int ndim, uint8_t* out, int64_t cap) {
  Writer w{out, out ? cap : 0};
  emit_header(w, shape, ndim);
  for (int64_t i = 0; i < count; ++i) emit_elem(w, ct + (size_t)i * n2w, n2w, exps[i], i, count);
  emit_footer(w);
  return w.n;
}

// ------------------------------------------------------------------ decoder
struct Val {
  enum Kind : uint8_t { NONE, BOOL, INT, BYTES, STR, TUPLE, LIST, DICT, GLOBAL, OBJ, MARK } k = NONE;
  bool neg = false;                 // INT sign
  int64_t off = -1, n = 0;          // payload (BYTES/STR bytes, non-negative INT magnitude) as a view of the input
  std::string s;                    // owned payload: negative INT magnitude, GLOBAL "module name"
  std::vector<int32_t> items;       // TUPLE/LIST elements, DICT key/value pairs
  int32_t cls = -1, args = -1, state = -1;  // OBJ: callable/class, its args, BUILD state
};

struct Machine {
  const uint8_t* p;
  int64_t len, pos = 0;
  std::vector<Val> arena;
  std::vector<int32_t> stack, memo;
  std::vector<size_t> marks;

  std::vector<int32_t> scratch;  // pop_mark result (reused: one element's SETITEMS at a time)

  explicit Machine(const uint8_t* d, int64_t l) : p(d), len(l) {
    arena.reserve((size_t)std::min<int64_t>(l / 64 + 64, (int64_t)1 << 26));
  }
  [[noreturn]] void bad(const char* why) { throw std::runtime_error(std::string("wire decode: ") + why); }
  const uint8_t* take(int64_t k) {
    if (k < 0 || k > len - pos) bad("truncated");  // no pos + k: k comes from an 8-byte field
    const uint8_t* r = p + pos;
    pos += k;
    return r;
  }
  uint64_t uint_le(int k) {
    const uint8_t* b = take(k);
    uint64_t v = 0;
    for (int i = 0; i < k; ++i) v |= (uint64_t)b[i] << (8 * i);
    return v;
  }
  int32_t make(Val v) {
    arena.push_back(std::move(v));
    return (int32_t)arena.size() - 1;
  }
  int32_t pop() {
    if (stack.empty() || (!marks.empty() && stack.size() <= marks.back())) bad("stack underflow");
    int32_t v = stack.back();
    stack.pop_back();
    return v;
  }
  const std::vector<int32_t>& pop_mark() {
    if (marks.empty()) bad("no mark");
    size_t m = marks.back();
    marks.pop_back();
    scratch.assign(stack.begin() + m, stack.end());
    stack.resize(m);
    return scratch;
  }
  // two's complement LE; `in_input`: b points into the pickle (kept as a view)
  int32_t make_int(const uint8_t* b, int64_t n, bool in_input) {
    Val v;
    v.k = Val::INT;
    if (n > 0 && (b[n - 1] & 0x80)) {  // negative: magnitude = -x
      v.neg = true;
      std::string m((const char*)b, (size_t)n);
      int carry = 1;
      for (auto& c : m) {
        int x = (uint8_t)~(uint8_t)c + carry;
        c = (char)(x & 0xff);
        carry = x >> 8;
      }
      v.s = m;
    } else if (in_input) {
      v.off = b - p;
      v.n = n;
    } else {
      v.s.assign((const char*)b, (size_t)n);
    }
    return make(std::move(v));
  }
  int32_t make_small(int64_t x) {
    uint8_t b[8];
    for (int i = 0; i < 8; ++i) b[i] = (uint8_t)((uint64_t)x >> (8 * i));
    return make_int(b, 8, false);
  }
  // payload bytes of a BYTES/STR/INT value
  std::string bytes_of(int32_t i) const {
    const Val& v = arena[i];
    return v.off >= 0 ? std::string((const char*)p + v.off, (size_t)v.n) : v.s;
  }
  bool str_eq(int32_t i, const char* lit) const {
    const Val& v = arena[i];
    size_t l = strlen(lit);
    if (v.off >= 0) return (size_t)v.n == l && memcmp(p + v.off, lit, l) == 0;
    return v.s == lit;
  }
  // the container an APPEND(S)/SETITEM(S)/BUILD writes into: the stack top,
  // which must exist and be of the right kind
  Val& target(Val::Kind want, const char* what) {
    if (stack.empty()) bad(what);
    Val& t = arena[stack.back()];
    if (t.k != want) bad(what);
    return t;
  }
  void put_memo(uint64_t i, int32_t v) {
    // a memo index never exceeds the number of values created (<= input bytes)
    if (i > (uint64_t)len || i > (1u << 26)) bad("memo index");
    if (memo.size() <= i) memo.resize(i + 1, -1);
    memo[i] = v;
  }
  int32_t get_memo(uint64_t i) {
    if (i >= memo.size() || memo[i] < 0) bad("memo miss");
    return memo[i];
  }
  std::string line() {
    int64_t s = pos;
    while (pos < len && p[pos] != '\n') ++pos;
    if (pos >= len) bad("truncated line");
    std::string r((const char*)p + s, (size_t)(pos - s));
    ++pos;
    return r;
  }

  int32_t run() {
    while (true) {
      uint8_t op = *take(1);
      switch (op) {
        case 0x80: take(1); break;                  // PROTO
        case 0x95: take(8); break;                  // FRAME (framing is transparent)
        case '.': return pop();                     // STOP
        case '(': marks.push_back(stack.size()); break;
        case ')': { Val v; v.k = Val::TUPLE; stack.push_back(make(v)); break; }
        case 't': { Val v; v.k = Val::TUPLE; v.items = pop_mark(); stack.push_back(make(std::move(v))); break; }
        case 0x85: case 0x86: case 0x87: {          // TUPLE1..3
          int k = op - 0x84;
          Val v;
          v.k = Val::TUPLE;
          v.items.resize(k);
          for (int i = k - 1; i >= 0; --i) v.items[i] = pop();
          stack.push_back(make(std::move(v)));
          break;
        }
        case ']': { Val v; v.k = Val::LIST; stack.push_back(make(v)); break; }
        case '}': { Val v; v.k = Val::DICT; stack.push_back(make(v)); break; }
        case 'a': {
          int32_t x = pop();
          target(Val::LIST, "append target").items.push_back(x);
          break;
        }
        case 'e': {
          const auto& xs = pop_mark();
          auto& l = target(Val::LIST, "appends target").items;
          l.insert(l.end(), xs.begin(), xs.end());
          break;
        }
        case 's': {
          int32_t v = pop(), k = pop();
          auto& d = target(Val::DICT, "setitem target").items;
          d.push_back(k);
          d.push_back(v);
          break;
        }
        case 'u': {
          const auto& xs = pop_mark();
          if (xs.size() % 2) bad("setitems");
          auto& d = target(Val::DICT, "setitems target").items;
          d.insert(d.end(), xs.begin(), xs.end());
          break;
        }
        case 'N': { Val v; stack.push_back(make(v)); break; }
        case 0x88: case 0x89: { Val v; v.k = Val::BOOL; v.neg = op == 0x88; stack.push_back(make(v)); break; }
        case 'J': stack.push_back(make_small((int32_t)uint_le(4))); break;
        case 'K': stack.push_back(make_small((int64_t)uint_le(1))); break;
        case 'M': stack.push_back(make_small((int64_t)uint_le(2))); break;
        case 0x8a: { int64_t n = (int64_t)uint_le(1); stack.push_back(make_int(take(n), n, true)); break; }
        case 0x8b: { int64_t n = (int64_t)(int32_t)uint_le(4); stack.push_back(make_int(take(n), n, true)); break; }
        case 0x8c: case 'X': case 0x8d: case 'C': case 'B': case 0x8e: {
          int lb = (op == 0x8c || op == 'C') ? 1 : (op == 'X' || op == 'B') ? 4 : 8;
          int64_t n = (int64_t)uint_le(lb);
          Val v;
          v.k = (op == 0x8c || op == 'X' || op == 0x8d) ? Val::STR : Val::BYTES;
          v.off = take(n) - p;
          v.n = n;
          stack.push_back(make(std::move(v)));
          break;
        }
        case 'G': { take(8); Val v; stack.push_back(make(v)); break; }  // BINFLOAT: not part of the format
        case 'c': {  // GLOBAL
          Val v;
          v.k = Val::GLOBAL;
          v.s = line();
          v.s += " " + line();
          stack.push_back(make(std::move(v)));
          break;
        }
        case 0x93: {  // STACK_GLOBAL
          int32_t name = pop(), mod = pop();
          if (arena[name].k != Val::STR || arena[mod].k != Val::STR) bad("stack_global");
          Val v;
          v.k = Val::GLOBAL;
          v.s = bytes_of(mod) + " " + bytes_of(name);
          stack.push_back(make(std::move(v)));
          break;
        }
        case 'R': case 0x81: {  // REDUCE / NEWOBJ
          int32_t args = pop(), cls = pop();
          Val v;
          v.k = Val::OBJ;
          v.cls = cls;
          v.args = args;
          stack.push_back(make(std::move(v)));
          break;
        }
        case 'b': {
          int32_t st = pop();
          target(Val::OBJ, "build target").state = st;
          break;
        }
        case 0x94: if (stack.empty()) bad("memoize"); put_memo(memo.size(), stack.back()); break;
        case 'q': if (stack.empty()) bad("binput"); put_memo(uint_le(1), stack.back()); break;
        case 'r': if (stack.empty()) bad("long_binput"); put_memo(uint_le(4), stack.back()); break;
        case 'h': stack.push_back(get_memo(uint_le(1))); break;
        case 'j': stack.push_back(get_memo(uint_le(4))); break;
        default: bad("unsupported opcode");
      }
    }
  }
};

inline bool is_global(const Machine& m, int32_t v, const char* mod_name) {
  return v >= 0 && m.arena[v].k == Val::GLOBAL && m.arena[v].s == mod_name;
}

// little-endian magnitude bytes -> n2w words (false if it does not fit)
inline bool mag_to_words(const std::string& mag, uint32_t* w, int n2w) {
  for (int i = 0; i < n2w; ++i) w[i] = 0;
  for (size_t i = 0; i < mag.size(); ++i) {
    uint8_t b = (uint8_t)mag[i];
    if (!b) continue;
    if (i / 4 >= (size_t)n2w) return false;
    w[i / 4] |= (uint32_t)b << (8 * (i % 4));
  }
  return true;
}

inline int32_t dict_get(const Machine& m, int32_t d, const char* key) {
  const auto& it = m.arena[d].items;
  for (size_t i = 0; i + 1 < it.size(); i += 2)
    if (m.arena[it[i]].k == Val::STR && m.str_eq(it[i], key)) return it[i + 1];
  return -1;
}

inline int64_t int_value(const Machine& m, int32_t v) {
  const Val& x = m.arena[v];
  if (x.k != Val::INT) throw std::runtime_error("wire decode: expected an int");
  std::string b = m.bytes_of(v);
  size_t n = b.size();
  while (n > 0 && b[n - 1] == 0) --n;
  if (n > 8) throw std::runtime_error("wire decode: int out of range");
  uint64_t u = 0;
  for (size_t i = 0; i < n; ++i) u |= (uint64_t)(uint8_t)b[i] << (8 * i);
  if (u > (uint64_t)INT64_MAX) throw std::runtime_error("wire decode: int out of range");
  return x.neg ? -(int64_t)u : (int64_t)u;
}


// Bytes of a header part / the first element's class+key strings, built once.
template <class F>
std::string emitted(F&& f) {
  Writer c{nullptr, 0};
  f(c);
  std::string s((size_t)c.n, '\0');
  Writer w{(uint8_t*)&s[0], c.n};
  f(w);
  return s;
}

// Fast path for the exact byte layout `encode` writes (what our peers send):
// one linear scan, a memcpy per value, no pickle machine. Returns -1 at the
// first deviation from that layout; decode() then runs the general machine,
// which accepts (or rejects) every other form of the same object graph.
inline int64_t decode_own(const uint8_t* p, int64_t len, int n2w, uint32_t* ct, int32_t* exps, int64_t cap_count,
                          int64_t* shape, int* ndim) {
  static const std::string A = emitted([](Writer& w) { emit_header_a(w); });
  static const std::string B = emitted([](Writer& w) { emit_header_b(w); });
  static const std::string CLS = emitted([](Writer& w) {
    w.str("common.crypto.paillier.paillier");
    w.str("RawCiphertext");
    w.put(0x93);
    w.put(0x94);
  });
  static const std::string VAL = emitted([](Writer& w) { w.str("value"); w.put(0x94); });
  static const std::string EXP = emitted([](Writer& w) { w.str("exp"); w.put(0x94); });
  int64_t pos = 0;
  auto lit = [&](const std::string& s) {
    if (len - pos < (int64_t)s.size() || memcmp(p + pos, s.data(), s.size()) != 0) return false;
    pos += (int64_t)s.size();
    return true;
  };
  auto byte = [&](uint8_t b) {
    if (pos < len && p[pos] == b) {
      ++pos;
      return true;
    }
    return false;
  };
  auto le = [&](int k, uint64_t* v) {
    if (len - pos < k) return false;
    uint64_t x = 0;
    for (int i = 0; i < k; ++i) x |= (uint64_t)p[pos + i] << (8 * i);
    pos += k;
    *v = x;
    return true;
  };
  if (!lit(A)) return -1;
  int nd = 0;
  while (pos < len && p[pos] != 't') {
    if (nd >= 8) return -1;
    uint64_t v;
    uint8_t op = p[pos++];
    if (op == 'K') {
      if (!le(1, &v)) return -1;
    } else if (op == 'J') {
      if (!le(4, &v)) return -1;
      v = (uint64_t)(int64_t)(int32_t)(uint32_t)v;
    } else if (op == 0x8a) {
      uint64_t k;
      if (!le(1, &k) || k != 8 || !le(8, &v)) return -1;
    } else {
      return -1;
    }
    shape[nd++] = (int64_t)v;
  }
  if (!lit(B)) return -1;
  int64_t i = 0;
  const int64_t wbytes = 4 * (int64_t)n2w;
  while (true) {
    if (i % 1000 == 0) {
      if (pos < len && p[pos] == 't') break;  // end of the list (no element opens a block here)
      if (!byte('(')) return -1;
    }
    if (i == 0 ? !lit(CLS) : !(byte('h') && byte(1))) return -1;
    if (!(byte(')') && byte(0x81) && byte('}') && byte('('))) return -1;
    if (i == 0 ? !lit(VAL) : !(byte('h') && byte(2))) return -1;
    uint64_t nb;
    if (byte(0x8a)) {
      if (!le(1, &nb)) return -1;
    } else if (byte(0x8b)) {
      if (!le(4, &nb)) return -1;
    } else {
      return -1;
    }
    if ((int64_t)nb > len - pos) return -1;
    const uint8_t* val = p + pos;
    pos += (int64_t)nb;
    int64_t used = (int64_t)nb;
    if (used > 0 && (val[used - 1] & 0x80)) return -1;  // negative: not a ciphertext
    while (used > 0 && val[used - 1] == 0) --used;
    if (used > wbytes) return -1;
    if (i == 0 ? !lit(EXP) : !(byte('h') && byte(3))) return -1;
    int64_t e;
    uint64_t v;
    if (byte('K')) {
      if (!le(1, &v)) return -1;
      e = (int64_t)v;
    } else if (byte('J')) {
      if (!le(4, &v)) return -1;
      e = (int64_t)(int32_t)(uint32_t)v;
    } else {
      return -1;
    }
    if (!(byte('u') && byte('b'))) return -1;
    if (i < cap_count) {
      uint8_t* row = (uint8_t*)(ct + (size_t)i * n2w);
      memcpy(row, val, (size_t)used);
      memset(row + used, 0, (size_t)(wbytes - used));
      exps[i] = (int32_t)e;
    }
    ++i;
    const bool closes = pos < len && p[pos] == 'e';
    if (closes) ++pos;
    if ((i % 1000 == 0) != closes) {  // a block of 1000 closes exactly at its end, or the list ends
      if (!closes || !(pos < len && p[pos] == 't')) return -1;
      break;
    }
    if (closes && i % 1000 != 0) break;
  }
  if (!(byte('t') && byte('b') && byte('.')) || pos != len) return -1;
  *ndim = nd;
  return i;
}

// Decodes into ct [count][n2w], exps [count]; shape/ndim of the array.
// Returns the element count; throws on any deviation from the format.
inline int64_t decode_general(const uint8_t* data, int64_t len, int n2w, uint32_t* ct, int32_t* exps,
                              int64_t cap_count, int64_t* shape, int* ndim) {
  Machine m(data, len);
  int32_t top = m.run();
  const Val& arr = m.arena[top];
  if (arr.k != Val::OBJ || arr.state < 0) throw std::runtime_error("wire decode: not an ndarray pickle");
  const Val& st = m.arena[arr.state];
  if (st.k != Val::TUPLE || st.items.size() != 5) throw std::runtime_error("wire decode: ndarray state");
  const Val& shp = m.arena[st.items[1]];
  const Val& lst = m.arena[st.items[4]];
  if (shp.k != Val::TUPLE || lst.k != Val::LIST || shp.items.size() > 8)
    throw std::runtime_error("wire decode: ndarray state");
  *ndim = (int)shp.items.size();
  for (int d = 0; d < *ndim; ++d) shape[d] = int_value(m, shp.items[d]);
  const int64_t count = (int64_t)lst.items.size();
  if (count > cap_count) return count;  // caller retries with room
  for (int64_t i = 0; i < count; ++i) {
    const Val& o = m.arena[lst.items[i]];
    if (o.k != Val::OBJ || o.state < 0 || !is_global(m, o.cls, "common.crypto.paillier.paillier RawCiphertext"))
      throw std::runtime_error("wire decode: element is not a RawCiphertext");
    int32_t val = dict_get(m, o.state, "value"), ex = dict_get(m, o.state, "exp");
    if (val < 0 || ex < 0) throw std::runtime_error("wire decode: RawCiphertext state");
    const Val* v = &m.arena[val];
    std::string mag;
    if (v->k == Val::INT) {
      if (v->neg) throw std::runtime_error("wire decode: negative ciphertext");
      mag = m.bytes_of(val);
    } else if (v->k == Val::OBJ && is_global(m, v->cls, "gmpy2 from_binary")) {
      const Val& a = m.arena[v->args];
      if (a.k != Val::TUPLE || a.items.size() != 1 || m.arena[a.items[0]].k != Val::BYTES)
        throw std::runtime_error("wire decode: gmpy2 value");
      const std::string b = m.bytes_of(a.items[0]);
      if (b.size() < 2 || (uint8_t)b[0] != 0x01) throw std::runtime_error("wire decode: gmpy2 binary type");
      if ((uint8_t)b[1] == 0x02) throw std::runtime_error("wire decode: negative ciphertext");
      mag = b.substr(2);
    } else {
      throw std::runtime_error("wire decode: value type");
    }
    if (!mag_to_words(mag, ct + (size_t)i * n2w, n2w)) throw std::runtime_error("wire decode: value too large");
    int64_t e = int_value(m, ex);
    if (e < INT32_MIN || e > INT32_MAX) throw std::runtime_error("wire decode: exponent range");
    exps[i] = (int32_t)e;
  }
  return count;
}

inline int64_t decode(const uint8_t* data, int64_t len, int n2w, uint32_t* ct, int32_t* exps, int64_t cap_count,
                      int64_t* shape, int* ndim) {
  const int64_t own = decode_own(data, len, n2w, ct, exps, cap_count, shape, ndim);
  if (own >= 0) return own;
  return decode_general(data, len, n2w, ct, exps, cap_count, shape, ndim);
}

}  // namespace wire
}  // namespace xhe
