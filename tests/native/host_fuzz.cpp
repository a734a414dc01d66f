// Sanitizer harness for the native host code that handles untrusted or
// arithmetic-critical input (built by tests/test_host_sanitize.py with
// g++ -fsanitize=address,undefined -fno-sanitize-recover=all):
//
//   host_fuzz wire SEED...   wire::decode (the peer-bytes pickle parser behind
//                            Paillier.ciphertext_from, paillier.py:260-271) on
//                            each seed, then on every truncation, on seeded
//                            random byte flips and opcode substitutions, and
//                            with every length / count field inflated; plus
//                            encode -> decode round trips of random vectors.
//                            A malformed input may only raise (runtime_error);
//                            any memory or UB error aborts under the sanitizers.
//   host_fuzz zstd           xhe_zstd_raw_frame / xhe_zstd_raw_extract (wire_abi.cpp,
//                            the framing of Paillier.serialize(compression=True)
//                            and the fast path of ciphertext_from): round trips
//                            at block-boundary sizes, then every truncation,
//                            header and block-header corruption and random
//                            flips of small frames; extract may only refuse.
//   host_fuzz bn             hostbn.hpp arithmetic (key setup, context.py:28-71)
//                            on lines "op a b m" (hex) from stdin, results to
//                            stdout for the Python side to check against int.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "../../include/xhe.h"
#include "../../xfl_amd/csrc/hostbn.hpp"
#include "../../xfl_amd/csrc/wire.hpp"

using Bytes = std::vector<uint8_t>;

static long g_ok = 0, g_rejected = 0;

static void try_decode(const Bytes& b, int n2w) {
  const int64_t cap = 8;  // the seeds hold <= 5 elements; a larger count is reported, not written
  static std::vector<uint32_t> ct((size_t)cap * 512);
  static std::vector<int32_t> ex(cap);
  int64_t shape[8];
  int ndim = 0;
  if (b.empty()) return;  // the C ABI rejects len <= 0 before decoding
  try {
    int64_t n = xhe::wire::decode(b.data(), (int64_t)b.size(), n2w, ct.data(), ex.data(), cap, shape, &ndim);
    if (n < 0) std::abort();
    ++g_ok;
  } catch (const std::runtime_error&) {
    ++g_rejected;
  }
}

static void fuzz_seed(const Bytes& seed, std::mt19937_64& rng) {
  const int n2ws[] = {128, 512};
  for (int n2w : n2ws) try_decode(seed, n2w);
  // every truncation
  for (size_t k = 0; k < seed.size(); ++k) try_decode(Bytes(seed.begin(), seed.begin() + k), 512);
  // random byte flips (1-3 bytes per mutant)
  for (int t = 0; t < 4000; ++t) {
    Bytes m = seed;
    int flips = 1 + (int)(rng() % 3);
    for (int f = 0; f < flips; ++f) m[rng() % m.size()] = (uint8_t)rng();
    try_decode(m, 512);
  }
  // opcode substitutions at every position
  static const uint8_t ops[] = {'a', 'e', 's', 'u', 'b', 't', ')', ']', '}', '(', 'R', 0x81, 0x93, 0x94, 'q',
                                'r', 'h', 'j', 0x85, 0x86, 0x87, 0x8a, 0x8b, 0x8c, 0x8d, 0x8e, 'B', 'C', 'X',
                                'K', 'M', 'J', 'N', '.', 0x80, 0x95, 'c', 'G', 0x88};
  for (size_t pos = 0; pos < seed.size(); ++pos) {
    Bytes m = seed;
    m[pos] = ops[rng() % sizeof(ops)];
    try_decode(m, 512);
  }
  // inflate every 1/4/8-byte little-endian field after a length-prefixed opcode
  for (size_t pos = 0; pos + 1 < seed.size(); ++pos) {
    uint8_t op = seed[pos];
    int lb = (op == 0x8c || op == 'C' || op == 0x8a || op == 'q' || op == 'h') ? 1
             : (op == 'X' || op == 'B' || op == 0x8b || op == 'r' || op == 'j') ? 4
             : (op == 0x8d || op == 0x8e || op == 0x95) ? 8 : 0;
    if (!lb || pos + 1 + lb > seed.size()) continue;
    static const uint64_t big[] = {~0ull, 0x7fffffffffffffffull, 0x8000000000000000ull, 0x7fffffffull,
                                   0xffffffffull, 0x80000000ull, 0xffull, 0x7full, 1ull << 40};
    for (uint64_t v : big) {
      Bytes m = seed;
      for (int i = 0; i < lb; ++i) m[pos + 1 + i] = (uint8_t)(v >> (8 * i));
      try_decode(m, 512);
    }
  }
}

static void crafted() {
  std::vector<Bytes> cases = {
      {'K', 1, 'a', '.'},                         // APPEND with no list under the value
      {']', 'K', 1, 'a', '.'},                    // well-formed append, bad top-level type
      {'K', 1, 'K', 2, 's', '.'},                 // SETITEM with no dict
      {')', 'K', 1, 'K', 2, 's', '.'},            // SETITEM into a tuple
      {'(', 'K', 1, 'e', '.'},                    // APPENDS with an empty stack under the mark
      {'K', 1, '(', 'K', 2, 'e', '.'},            // APPENDS into an int
      {'K', 1, '}', 'b', '.'},                    // BUILD on a dict
      {'}', 'b', '.'},                            // BUILD with nothing under the state
      {'.'},                                      // STOP on an empty stack
      {0x94},                                     // MEMOIZE on an empty stack
      {'h', 0, '.'},                              // memo miss
      {'r', 0xff, 0xff, 0xff, 0x7f, '.'},         // LONG_BINPUT with an empty stack
      {'K', 1, 'r', 0xff, 0xff, 0xff, 0x03, '.'}, // memo index 2^26-1 from a 9-byte input
      {0x8e, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f, 'x'},  // BINBYTES8 of length INT64_MAX
      {0x8d, 0xf0, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f, 'x'},  // BINUNICODE8 near INT64_MAX
      {0x8b, 0xff, 0xff, 0xff, 0xff},             // LONG4 with a negative length
      {'c', 'a'},                                 // GLOBAL without newline
      {0x93, '.'},                                // STACK_GLOBAL on an empty stack
      {'K', 1, 'K', 2, 0x93, '.'},                // STACK_GLOBAL of non-strings
      {'R', '.'},                                 // REDUCE underflow
      {0x85, '.'},                                // TUPLE1 underflow
      {'(', '(', '(', 't', 't', 't', 't', '.'},   // pop_mark without a mark
  };
  for (auto& c : cases) try_decode(c, 128);
}

static void roundtrip(std::mt19937_64& rng) {
  for (int t = 0; t < 200; ++t) {
    const int n2w = (t % 2) ? 128 : 512;
    const int64_t count = (int64_t)(rng() % 9);
    std::vector<uint32_t> ct((size_t)std::max<int64_t>(count, 1) * n2w);
    std::vector<int32_t> ex((size_t)std::max<int64_t>(count, 1));
    for (auto& w : ct) w = (rng() % 4 == 0) ? 0u : (uint32_t)rng();
    for (auto& e : ex) e = (int32_t)rng();
    if (count) ct[(size_t)(count - 1) * n2w + n2w - 1] = 0;  // a value with leading zero words
    int64_t shape[2] = {count, 1};
    int64_t need = xhe::wire::encode(ct.data(), ex.data(), count, n2w, shape, 2, nullptr, 0);
    Bytes out((size_t)need);
    if (xhe::wire::encode(ct.data(), ex.data(), count, n2w, shape, 2, out.data(), need) != need) std::abort();
    std::vector<uint32_t> ct2(ct.size(), 0xdeadbeef);
    std::vector<int32_t> ex2(ex.size(), 0);
    int64_t shp[8];
    int nd = 0;
    int64_t n = xhe::wire::decode(out.data(), need, n2w, ct2.data(), ex2.data(), std::max<int64_t>(count, 1), shp,
                                  &nd);
    if (n != count || nd != 2 || shp[0] != count || shp[1] != 1) std::abort();
    for (int64_t i = 0; i < count; ++i) {
      if (ex2[i] != ex[i]) std::abort();
      if (std::memcmp(&ct2[(size_t)i * n2w], &ct[(size_t)i * n2w], (size_t)n2w * 4)) std::abort();
    }
  }
}

// Our own encoder's output: the fast decode path must accept it and agree
// with the general pickle machine; then it is fuzzed like the other seeds.
static void own_format(std::mt19937_64& rng) {
  const int64_t counts[] = {0, 1, 5, 999, 1000, 1001, 2500, 9001};
  for (int64_t count : counts) {
    const int n2w = 128;
    std::vector<uint32_t> ct((size_t)std::max<int64_t>(count, 1) * n2w);
    std::vector<int32_t> ex((size_t)std::max<int64_t>(count, 1));
    for (auto& w : ct) w = (uint32_t)rng();
    for (int64_t i = 0; i < count; ++i) {
      ex[i] = (int32_t)(rng() % 3 == 0 ? rng() : rng() % 300);
      int top = (int)(rng() % n2w);  // varying value lengths, incl. LONG1/LONG4 and zero
      for (int k = top; k < n2w; ++k) ct[(size_t)i * n2w + k] = 0;
    }
    int64_t shape[2] = {count, 1};
    for (int threads : {1, 3, 16}) {
      int64_t need = xhe::wire::encode(ct.data(), ex.data(), count, n2w, shape, 2, nullptr, 0, threads);
      Bytes out((size_t)need);
      xhe::wire::encode(ct.data(), ex.data(), count, n2w, shape, 2, out.data(), need, threads);
      Bytes ref((size_t)xhe::wire::encode_reference(ct.data(), ex.data(), count, n2w, shape, 2, nullptr, 0));
      xhe::wire::encode_reference(ct.data(), ex.data(), count, n2w, shape, 2, ref.data(), (int64_t)ref.size());
      if (ref != out) std::abort();  // the fast writer produces the specification's bytes
      // the one-pass writer (encode_to) through a plain sink, and through a
      // framed sink with small blocks (payloads split across block borders)
      {
        Bytes flat((size_t)need);
        const xhe::wire::Sink plain{flat.data(), 0};
        if (xhe::wire::encode_to(ct.data(), ex.data(), count, n2w, shape, 2, &plain, threads) != need) std::abort();
        if (flat != out) std::abort();
        // layout from bit lengths + rows in chunks (the serialize pipeline)
        std::vector<int16_t> bits((size_t)std::max<int64_t>(count, 1), 0);
        for (int64_t i = 0; i < count; ++i) {
          int k = n2w - 1;
          while (k >= 0 && ct[(size_t)i * n2w + k] == 0) --k;
          bits[i] = (int16_t)(k < 0 ? 0 : 32 * k + 32 - __builtin_clz(ct[(size_t)i * n2w + k]));
        }
        std::vector<int64_t> offs((size_t)count + 1);
        Bytes piece((size_t)need, 0xEE);
        const xhe::wire::Sink ps{piece.data(), 0};
        if (xhe::wire::layout(bits.data(), ex.data(), count, n2w, shape, 2, offs.data(), &ps, threads) != need)
          std::abort();
        for (int64_t lo = 0; lo < count; lo += 777) {
          const int64_t hi = std::min<int64_t>(count, lo + 777);
          if (!xhe::wire::write_rows(ct.data() + (size_t)lo * n2w, ex.data(), lo, hi, count, n2w, offs.data(), ps,
                                     threads))
            std::abort();
        }
        if (piece != out) std::abort();
        {  // the same range by range (the pipeline over a running encryption):
           // header, per-range offsets from the previous range's end, rows, footer
          std::vector<int64_t> o2((size_t)count + 1, -1);
          Bytes inc((size_t)need + 4096, 0xEE);  // over-allocated, as the caller does
          const xhe::wire::Sink is{inc.data(), 0};
          o2[0] = xhe::wire::head_bytes(shape, 2);
          xhe::wire::write_head(shape, 2, is);
          for (int64_t lo = 0; lo < count; lo += 1000) {
            const int64_t hi = std::min<int64_t>(count, lo + 1000);
            if ((lo / 1000) % 2)
              xhe::wire::layout_part_rows(ct.data() + (size_t)lo * n2w, ex.data(), lo, hi, count, n2w, o2.data());
            else
              xhe::wire::layout_part(bits.data() + lo, ex.data(), lo, hi, count, n2w, o2.data());
            if (!xhe::wire::write_rows(ct.data() + (size_t)lo * n2w, ex.data(), lo, hi, count, n2w, o2.data(), is,
                                       threads))
              std::abort();
          }
          xhe::wire::write_foot(o2[count], is);
          if (o2[count] + 3 != need || o2 != offs) std::abort();
          // one range over several threads gives the same offsets
          std::vector<int64_t> o3((size_t)count + 1, -1);
          o3[0] = o2[0];
          xhe::wire::layout_part_rows(ct.data(), ex.data(), 0, count, count, n2w, o3.data(), threads);
          if (o3 != offs) std::abort();
          if (std::memcmp(inc.data(), out.data(), (size_t)need)) std::abort();
        }
        if (count > 1) {  // a wrong bit length is refused
          bits[1] = (int16_t)(bits[1] > 8 ? bits[1] - 8 : bits[1] + 8);
          xhe::wire::layout(bits.data(), ex.data(), count, n2w, shape, 2, offs.data(), nullptr, threads);
          if (xhe::wire::write_rows(ct.data(), ex.data(), 0, count, count, n2w, offs.data(), ps, threads)) std::abort();
        }
        for (int64_t blk : {(int64_t)1, (int64_t)37, (int64_t)1000, (int64_t)131072}) {
          const int64_t nbk = (need + blk - 1) / blk;
          Bytes fr((size_t)(14 + need + 3 * nbk), 0xEE);
          const xhe::wire::Sink framed{fr.data(), blk};
          xhe::wire::encode_to(ct.data(), ex.data(), count, n2w, shape, 2, &framed, threads);
          for (int64_t b = 0; b < nbk; ++b) {
            const int64_t len = std::min<int64_t>(blk, need - b * blk);
            const uint8_t* pay = fr.data() + 14 + b * (blk + 3) + 3;
            if (std::memcmp(pay, out.data() + b * blk, (size_t)len)) std::abort();
            for (int k = 0; k < 3; ++k)  // block headers untouched (the caller writes them)
              if (fr[(size_t)(14 + b * (blk + 3) + k)] != 0xEE) std::abort();
          }
        }
      }
      const int64_t cap = std::max<int64_t>(count, 1);
      std::vector<uint32_t> a((size_t)cap * n2w), b((size_t)cap * n2w);
      std::vector<int32_t> ea(cap), eb(cap);
      int64_t sa[8], sb[8];
      int na = 0, nb = 0;
      int64_t ka = xhe::wire::decode_own(out.data(), need, n2w, a.data(), ea.data(), cap, sa, &na);
      int64_t kb = xhe::wire::decode_general(out.data(), need, n2w, b.data(), eb.data(), cap, sb, &nb);
      if (ka != count || kb != count || na != 2 || nb != 2 || sa[0] != count || sb[0] != count) std::abort();
      if (count && (a != b || ea != eb)) std::abort();
      if (count && std::memcmp(a.data(), ct.data(), (size_t)count * n2w * 4)) std::abort();
      if (count > 0 && count <= 5) fuzz_seed(out, rng);
    }
  }
}

static xhe::BigU from_hex(const std::string& h) {
  std::vector<uint32_t> w((h.size() + 7) / 8 + 1, 0);
  int bit = 0;
  for (int i = (int)h.size() - 1; i >= 0; --i, bit += 4) {
    char c = h[i];
    uint32_t v = (c >= '0' && c <= '9') ? c - '0' : (c | 32) - 'a' + 10;
    w[bit / 32] |= v << (bit % 32);
  }
  return xhe::BigU::from_words(w.data(), w.size());
}

static void print_hex(const xhe::BigU& a) {
  if (a.is_zero()) {
    std::printf("0\n");
    return;
  }
  std::printf("%x", a.w.back());
  for (size_t i = a.w.size() - 1; i-- > 0;) std::printf("%08x", a.w[i]);
  std::printf("\n");
}

static int bn_mode() {
  std::string op, as, bs, ms;
  while (std::cin >> op >> as >> bs >> ms) {
    xhe::BigU a = from_hex(as), b = from_hex(bs), m = from_hex(ms);
    try {
      if (op == "add") print_hex(xhe::add(a, b));
      else if (op == "sub") print_hex(xhe::sub(a, b));
      else if (op == "mul") print_hex(xhe::mul(a, b));
      else if (op == "mod") print_hex(xhe::mod(a, m));
      else if (op == "mulmod") print_hex(xhe::mulmod(a, b, m));
      else if (op == "powmod") print_hex(xhe::powmod(a, b, m));
      else if (op == "modinv") print_hex(xhe::modinv(a, m));
      else if (op == "ninv") std::printf("%x\n", xhe::mont_ninv(m.word(0), (int)a.word(0)));
      else if (op == "words_inv") {
        const int nw = (int)m.w.size();
        std::vector<uint32_t> x(nw), mm(nw), y(nw);
        a.to_words(x.data(), nw);
        m.to_words(mm.data(), nw);
        if (xhe::modinv_words(x.data(), mm.data(), nw, y.data())) print_hex(xhe::BigU::from_words(y.data(), nw));
        else std::printf("none\n");
      } else std::printf("?\n");
    } catch (const std::runtime_error&) {
      std::printf("error\n");
    }
  }
  return 0;
}

static int zstd_mode() {
  std::mt19937_64 rng(777);
  long frames = 0, refused = 0;
  const int64_t B = 1 << 17;
  const int64_t sizes[] = {0, 1, 2, 1000, B - 1, B, B + 1, 3 * B, 5 * B + 17, (8 << 20) + 3};
  auto extract = [&](const Bytes& f, int64_t cap) -> int {
    int64_t n = 0;
    Bytes out((size_t)std::max<int64_t>(cap, 1));
    int rc = xhe_zstd_raw_extract(f.empty() ? nullptr : f.data(), (int64_t)f.size(), cap ? out.data() : nullptr, cap,
                                  &n);
    if (rc != XHE_OK && rc != XHE_ENOTSUP && rc != XHE_EOVERFLOW && rc != XHE_EINVAL) std::abort();
    if (rc != XHE_OK) ++refused;
    return rc;
  };
  for (int64_t n : sizes) {
    Bytes src((size_t)n);
    for (auto& b : src) b = (uint8_t)rng();
    const int64_t size = xhe_zstd_raw_frame_size(n);
    Bytes f((size_t)size);
    int64_t got = 0;
    if (xhe_zstd_raw_frame(n ? src.data() : nullptr, n, f.data(), size, &got) != XHE_OK || got != size) std::abort();
    if (xhe_zstd_raw_frame(n ? src.data() : nullptr, n, f.data(), size - 1, &got) != XHE_EOVERFLOW) std::abort();
    ++frames;
    Bytes back((size_t)std::max<int64_t>(n, 1));
    int64_t m = -1;
    if (xhe_zstd_raw_extract(f.data(), size, back.data(), n, &m) != XHE_OK || m != n) std::abort();
    if (n && std::memcmp(back.data(), src.data(), (size_t)n)) std::abort();
    if (n > 4 * B) continue;  // mutate the small frames only
    for (int64_t k = 0; k < size; k += (k < 64 ? 1 : 997)) extract(Bytes(f.begin(), f.begin() + k), n);
    for (int64_t pos = 0; pos < std::min<int64_t>(size, 32); ++pos)
      for (int v : {0x00, 0x01, 0x04, 0x20, 0x40, 0x80, 0xC0, 0xFF}) {
        Bytes g = f;
        g[pos] = (uint8_t)v;
        extract(g, n);
        extract(g, n + 4096);
      }
    for (int t = 0; t < 300; ++t) {
      Bytes g = f;
      g[rng() % g.size()] = (uint8_t)rng();
      extract(g, n);
    }
  }
  std::printf("zstd frames %ld refused %ld\n", frames, refused);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "bn") return bn_mode();
  if (argc >= 2 && std::string(argv[1]) == "zstd") return zstd_mode();
  if (argc < 3 || std::string(argv[1]) != "wire") {
    std::fprintf(stderr, "usage: host_fuzz wire SEED... | host_fuzz bn < cases\n");
    return 2;
  }
  std::mt19937_64 rng(12345);
  long seeds_ok = 0;
  for (int i = 2; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    Bytes seed((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    long before = g_ok;
    try_decode(seed, 512);
    if (g_ok == before) {
      std::fprintf(stderr, "seed %s did not decode\n", argv[i]);
      return 1;
    }
    ++seeds_ok;
    fuzz_seed(seed, rng);
  }
  crafted();
  roundtrip(rng);
  own_format(rng);
  std::printf("seeds %ld decoded %ld rejected %ld\n", seeds_ok, g_ok, g_rejected);
  return 0;
}
