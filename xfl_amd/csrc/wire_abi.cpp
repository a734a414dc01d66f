// Host-only part of the xhe C ABI (include/xhe.h): the wire codec entry
// points and the error channel. Compiled by the host compiler and linked into
// libxhe.so next to xhe.hip's object, so codec changes rebuild in seconds.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "../../include/xhe.h"
#include "abi_common.hpp"
#include "wire.hpp"

namespace {
thread_local std::string g_err;

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::exception& e) {
    return xhe_fail(XHE_EINVAL, e.what());
  }
}

// host threads for the codec: the machine's cores, at most 16 (a GPU box's
// CPU share per GPU)
constexpr int kZstdWindowLog = 17;
constexpr int64_t kZstdBlock = (int64_t)1 << kZstdWindowLog;  // = the format's 128 KiB block maximum

int codec_threads() {
  unsigned hc = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(hc ? hc : 1u, 16u));
}
}  // namespace

int xhe_fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

void xhe_host_copy(void* dst, const void* src, int64_t n) {
  if (n <= 0) return;
  const int T = n >= (8 << 20) ? codec_threads() : 1;
  const int64_t per = ((n + T - 1) / T + 4095) & ~(int64_t)4095;
  xhe::wire::run_parallel(T, [&](int t) {
    const int64_t lo = (int64_t)t * per, hi = std::min<int64_t>(n, lo + per);
    if (hi > lo) memcpy(static_cast<uint8_t*>(dst) + lo, static_cast<const uint8_t*>(src) + lo, hi - lo);
  });
}

extern "C" {

int xhe_host_prefault(void* p, int64_t nbytes) {
  // One write per 4 KiB page, the range split over the codec threads: the
  // kernel's zero-fill of fresh pages then runs on all of them instead of
  // inside the single thread that later copies device results in.
  if (!p || nbytes < 0) return xhe_fail(XHE_EINVAL, "xhe_host_prefault: bad argument");
  const int T = nbytes >= (64 << 20) ? codec_threads() : 1;
  auto* base = static_cast<volatile uint8_t*>(p);
  const int64_t per = ((nbytes + T - 1) / T + 4095) & ~(int64_t)4095;
  xhe::wire::run_parallel(T, [&](int t) {
    const int64_t lo = (int64_t)t * per, hi = std::min<int64_t>(nbytes, lo + per);
    for (int64_t o = lo; o < hi; o += 4096) base[o] = 0;
  });
  return XHE_OK;
}

int64_t xhe_zstd_raw_frame_size(int64_t n) {
  const int64_t nb = n > 0 ? (n + kZstdBlock - 1) / kZstdBlock : 1;
  return 14 + n + 3 * nb;
}

int xhe_zstd_raw_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* out_len) {
  // One zstd frame (RFC 8878) holding `src` as raw blocks: magic, a frame
  // header with an 8-byte content size and a 128 KiB window (not single-
  // segment, so streaming decoders need no content-sized window), then
  // ceil(n / 128 KiB) raw blocks, the last one flagged. The layout is known
  // in closed form, so the blocks are written by all codec threads at once.
  if (!out_len || n < 0 || (n > 0 && !src)) return xhe_fail(XHE_EINVAL, "xhe_zstd_raw_frame: bad argument");
  const int64_t need = xhe_zstd_raw_frame_size(n);
  *out_len = need;
  if (!dst || cap < need) return xhe_fail(XHE_EOVERFLOW, "xhe_zstd_raw_frame: output buffer too small");
  static const uint8_t head[6] = {0x28, 0xB5, 0x2F, 0xFD, 0xC0, (uint8_t)((kZstdWindowLog - 10) << 3)};
  memcpy(dst, head, 6);
  for (int k = 0; k < 8; ++k) dst[6 + k] = (uint8_t)((uint64_t)n >> (8 * k));
  const int64_t nb = n > 0 ? (n + kZstdBlock - 1) / kZstdBlock : 1;
  const int T = n >= (8 << 20) ? codec_threads() : 1;
  xhe::wire::run_parallel(T, [&](int t) {
    for (int64_t b = nb * t / T; b < nb * (t + 1) / T; ++b) {
      const int64_t lo = b * kZstdBlock, len = std::min<int64_t>(kZstdBlock, n - lo);
      uint8_t* o = dst + 14 + b * (kZstdBlock + 3);
      const uint32_t h = (uint32_t)(b == nb - 1) | (0u << 1) | ((uint32_t)len << 3);  // Last_Block, Raw, Block_Size
      o[0] = (uint8_t)h;
      o[1] = (uint8_t)(h >> 8);
      o[2] = (uint8_t)(h >> 16);
      if (len > 0) memcpy(o + 3, src + lo, len);
    }
  });
  return XHE_OK;
}

int xhe_zstd_raw_extract(const uint8_t* src, int64_t len, uint8_t* dst, int64_t cap, int64_t* out_len) {
  // The inverse for frames made only of raw blocks (what xhe_zstd_raw_frame
  // writes): walk the block headers, then copy the payloads in parallel.
  // Anything else - compressed or RLE blocks, a content checksum, a
  // dictionary, trailing data, a missing content size - is XHE_ENOTSUP and
  // left to libzstd.
  if (!out_len || len < 0 || (len > 0 && !src)) return xhe_fail(XHE_EINVAL, "xhe_zstd_raw_extract: bad argument");
  *out_len = -1;
  auto unsup = [] { return xhe_fail(XHE_ENOTSUP, "not a raw-block zstd frame"); };
  if (len < 6 || src[0] != 0x28 || src[1] != 0xB5 || src[2] != 0x2F || src[3] != 0xFD) return unsup();
  const uint8_t fhd = src[4];
  const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1;
  if ((fhd & 0x0F) != 0) return unsup();  // reserved bit, checksum or dictionary id
  const int fcs_bytes = fcs_flag == 0 ? (single ? 1 : 0) : (1 << fcs_flag);
  if (fcs_bytes == 0) return unsup();
  int64_t pos = 5 + (single ? 0 : 1);
  if (pos + fcs_bytes > len) return unsup();
  uint64_t fcs = 0;
  for (int k = 0; k < fcs_bytes; ++k) fcs |= (uint64_t)src[pos + k] << (8 * k);
  if (fcs_bytes == 2) fcs += 256;
  pos += fcs_bytes;
  if (fcs > (uint64_t)INT64_MAX) return unsup();
  std::vector<int64_t> from, to, size;
  int64_t outp = 0;
  for (bool last = false; !last;) {
    if (pos + 3 > len) return unsup();
    const uint32_t h = src[pos] | ((uint32_t)src[pos + 1] << 8) | ((uint32_t)src[pos + 2] << 16);
    last = h & 1;
    const int64_t bs = h >> 3;
    pos += 3;
    if (((h >> 1) & 3) != 0 || bs > len - pos || bs > (int64_t)fcs - outp) return unsup();
    from.push_back(pos);
    to.push_back(outp);
    size.push_back(bs);
    pos += bs;
    outp += bs;
  }
  if (pos != len || outp != (int64_t)fcs) return unsup();
  *out_len = outp;
  if (!dst || cap < outp) return xhe_fail(XHE_EOVERFLOW, "xhe_zstd_raw_extract: output buffer too small");
  const int64_t nb = (int64_t)from.size();
  const int T = outp >= (8 << 20) ? codec_threads() : 1;
  xhe::wire::run_parallel(T, [&](int t) {
    for (int64_t b = nb * t / T; b < nb * (t + 1) / T; ++b)
      if (size[b]) memcpy(dst + to[b], src + from[b], size[b]);
  });
  return XHE_OK;
}

int xhe_wire_encode(const uint32_t* ct, const int32_t* exps, int64_t count, int n2w, const int64_t* shape, int ndim,
                    uint8_t* out, int64_t cap, int64_t* out_len) {
  return guarded([&]() -> int {
    if (!out_len || count < 0 || n2w <= 0 || ndim < 0 || ndim > 8 || (count > 0 && (!ct || !exps)) ||
        (ndim > 0 && !shape))
      return xhe_fail(XHE_EINVAL, "xhe_wire_encode: bad argument");
    int64_t prod = 1;
    for (int d = 0; d < ndim; ++d) prod *= shape[d];
    if (prod != count) return xhe_fail(XHE_EINVAL, "xhe_wire_encode: shape does not match count");
    int64_t need = xhe::wire::encode(ct, exps, count, n2w, shape, ndim, out, out ? cap : 0, codec_threads());
    *out_len = need;
    if (!out || need > cap) return xhe_fail(XHE_EOVERFLOW, "xhe_wire_encode: output buffer too small");
    return XHE_OK;
  });
}

namespace {
// frame header + every block header of a raw-block frame holding pk content bytes
void write_frame_headers(uint8_t* out, int64_t pk) {
  static const uint8_t head[6] = {0x28, 0xB5, 0x2F, 0xFD, 0xC0, (uint8_t)((kZstdWindowLog - 10) << 3)};
  memcpy(out, head, 6);
  for (int k = 0; k < 8; ++k) out[6 + k] = (uint8_t)((uint64_t)pk >> (8 * k));
  const int64_t nb = (pk + kZstdBlock - 1) / kZstdBlock;
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t len = std::min<int64_t>(kZstdBlock, pk - b * kZstdBlock);
    const uint32_t h = (uint32_t)(b == nb - 1) | ((uint32_t)len << 3);  // Last_Block, Raw, Block_Size
    uint8_t* o = out + 14 + b * (kZstdBlock + 3);
    o[0] = (uint8_t)h;
    o[1] = (uint8_t)(h >> 8);
    o[2] = (uint8_t)(h >> 16);
  }
}
}  // namespace

int xhe_wire_encode_frame(const uint32_t* ct, const int32_t* exps, int64_t count, int n2w, const int64_t* shape,
                          int ndim, int framed, uint8_t* out, int64_t cap, int64_t* out_len) {
  return guarded([&]() -> int {
    if (!out_len || count < 0 || n2w <= 0 || ndim < 0 || ndim > 8 || (count > 0 && (!ct || !exps)) ||
        (ndim > 0 && !shape))
      return xhe_fail(XHE_EINVAL, "xhe_wire_encode_frame: bad argument");
    int64_t prod = 1;
    for (int d = 0; d < ndim; ++d) prod *= shape[d];
    if (prod != count) return xhe_fail(XHE_EINVAL, "xhe_wire_encode_frame: shape does not match count");
    const int T = codec_threads();
    const int64_t pk = xhe::wire::encode_to(ct, exps, count, n2w, shape, ndim, nullptr, T);
    const int64_t need = framed ? xhe_zstd_raw_frame_size(pk) : pk;
    *out_len = need;
    if (!out || need > cap) return xhe_fail(XHE_EOVERFLOW, "xhe_wire_encode_frame: output buffer too small");
    if (framed) write_frame_headers(out, pk);  // those of xhe_zstd_raw_frame(pickle); the pickle into the payloads
    const xhe::wire::Sink sink{out, framed ? kZstdBlock : 0};
    xhe::wire::encode_to(ct, exps, count, n2w, shape, ndim, &sink, T);
    return XHE_OK;
  });
}

int xhe_wire_layout(const int16_t* bits, const int32_t* exps, int64_t count, int n2w, const int64_t* shape, int ndim,
                    int framed, int64_t* elem_off, uint8_t* out, int64_t cap, int64_t* out_len) {
  return guarded([&]() -> int {
    if (!out_len || !elem_off || count < 0 || n2w <= 0 || n2w > 1023 || ndim < 0 || ndim > 8 ||
        (count > 0 && (!bits || !exps)) || (ndim > 0 && !shape))
      return xhe_fail(XHE_EINVAL, "xhe_wire_layout: bad argument");
    int64_t prod = 1;
    for (int d = 0; d < ndim; ++d) prod *= shape[d];
    if (prod != count) return xhe_fail(XHE_EINVAL, "xhe_wire_layout: shape does not match count");
    for (int64_t i = 0; i < count; ++i)
      if (bits[i] < 0 || bits[i] > 32 * n2w) return xhe_fail(XHE_EINVAL, "xhe_wire_layout: bit length out of range");
    const int T = codec_threads();
    const int64_t pk = xhe::wire::layout(bits, exps, count, n2w, shape, ndim, elem_off, nullptr, T);
    const int64_t need = framed ? xhe_zstd_raw_frame_size(pk) : pk;
    *out_len = need;
    if (!out) return XHE_OK;
    if (need > cap) return xhe_fail(XHE_EOVERFLOW, "xhe_wire_layout: output buffer too small");
    if (framed) write_frame_headers(out, pk);
    const xhe::wire::Sink sink{out, framed ? kZstdBlock : 0};
    xhe::wire::layout(bits, exps, count, n2w, shape, ndim, elem_off, &sink, T);
    return XHE_OK;
  });
}

int xhe_wire_rows(const uint32_t* rows, const int32_t* exps, int64_t lo, int64_t hi, int64_t count, int n2w,
                  const int64_t* elem_off, int framed, uint8_t* out, int64_t cap) {
  return guarded([&]() -> int {
    if (!rows || !exps || !elem_off || !out || lo < 0 || hi < lo || hi > count || n2w <= 0 || n2w > 1023)
      return xhe_fail(XHE_EINVAL, "xhe_wire_rows: bad argument");
    // the rows' last byte must fit (elem_off[count] may not be known yet: the
    // incremental layout fills the offsets range by range)
    const int64_t end = elem_off[hi];
    if (elem_off[lo] < 0 || end < elem_off[lo] || (framed ? xhe_zstd_raw_frame_size(end) : end) > cap)
      return xhe_fail(XHE_EOVERFLOW, "xhe_wire_rows: output buffer smaller than the layout");
    const xhe::wire::Sink sink{out, framed ? kZstdBlock : 0};
    if (!xhe::wire::write_rows(rows, exps, lo, hi, count, n2w, elem_off, sink, codec_threads()))
      return xhe_fail(XHE_EINVAL, "xhe_wire_rows: a row's bit length differs from the layout's");
    return XHE_OK;
  });
}

int xhe_wire_begin(const int32_t* exps, int64_t count, int n2w, const int64_t* shape, int ndim, int framed,
                   int64_t* elem_off, int64_t* max_len, uint8_t* out, int64_t cap) {
  return guarded([&]() -> int {
    if (!elem_off || !max_len || count < 0 || n2w <= 0 || n2w > 1023 || ndim < 0 || ndim > 8 ||
        (count > 0 && !exps) || (ndim > 0 && !shape))
      return xhe_fail(XHE_EINVAL, "xhe_wire_begin: bad argument");
    int64_t prod = 1;
    for (int d = 0; d < ndim; ++d) prod *= shape[d];
    if (prod != count) return xhe_fail(XHE_EINVAL, "xhe_wire_begin: shape does not match count");
    const int64_t head = xhe::wire::head_bytes(shape, ndim);
    // every element at the largest bit length its words allow, in closed form
    // (a call per element cost ~5 ms per 1 M, twice per serialize): element 0
    // exactly, the others at the small-exponent size, + 3 bytes per exponent
    // outside [0, 256) (BININT vs BININT1), + the APPENDS marks
    int64_t pk = head + 3;
    if (count > 0) {
      const int bits = 32 * n2w;
      pk += xhe::wire::elem_bytes_bits(bits, n2w, exps[0], 0, count);
      const int64_t nb = (bits + 8) / 8;
      const int64_t base = 8 + (nb < 256 ? 2 : 5) + nb + 2 + 2 + 2;
      int64_t wide = 0;
      for (int64_t i = 1; i < count; ++i) wide += (exps[i] < 0 || exps[i] >= 256) ? 1 : 0;
      const int64_t marks_open = (count - 1) / 1000;                   // i % 1000 == 0, i >= 1
      const int64_t marks_close = (count >= 1000 ? (count - 1000) / 1000 + 1 : 0) -
                                  ((count - 1) % 1000 == 999 ? 1 : 0) + (count > 1 ? 1 : 0);
      pk += (count - 1) * base + 3 * wide + marks_open + marks_close;
    }
    elem_off[0] = head;
    *max_len = framed ? xhe_zstd_raw_frame_size(pk) : pk;
    if (!out) return XHE_OK;
    if (*max_len > cap) return xhe_fail(XHE_EOVERFLOW, "xhe_wire_begin: output buffer too small");
    xhe::wire::write_head(shape, ndim, xhe::wire::Sink{out, framed ? kZstdBlock : 0});
    return XHE_OK;
  });
}

int xhe_wire_layout_part(const int16_t* bits, const int32_t* exps, int64_t lo, int64_t hi, int64_t count, int n2w,
                         int64_t* elem_off) {
  return guarded([&]() -> int {
    if (!elem_off || lo < 0 || hi < lo || hi > count || n2w <= 0 || n2w > 1023 || (hi > lo && (!bits || !exps)))
      return xhe_fail(XHE_EINVAL, "xhe_wire_layout_part: bad argument");
    for (int64_t i = 0; i < hi - lo; ++i)
      if (bits[i] < 0 || bits[i] > 32 * n2w)
        return xhe_fail(XHE_EINVAL, "xhe_wire_layout_part: bit length out of range");
    xhe::wire::layout_part(bits, exps, lo, hi, count, n2w, elem_off);
    return XHE_OK;
  });
}

int xhe_wire_layout_part_rows(const uint32_t* rows, const int32_t* exps, int64_t lo, int64_t hi, int64_t count,
                              int n2w, int64_t* elem_off) {
  return guarded([&]() -> int {
    if (!elem_off || lo < 0 || hi < lo || hi > count || n2w <= 0 || n2w > 1023 || (hi > lo && (!rows || !exps)))
      return xhe_fail(XHE_EINVAL, "xhe_wire_layout_part_rows: bad argument");
    xhe::wire::layout_part_rows(rows, exps, lo, hi, count, n2w, elem_off, codec_threads());
    return XHE_OK;
  });
}

int xhe_wire_finish(int64_t count, const int64_t* elem_off, int framed, uint8_t* out, int64_t cap, int64_t* out_len) {
  return guarded([&]() -> int {
    if (!elem_off || !out || !out_len || count < 0) return xhe_fail(XHE_EINVAL, "xhe_wire_finish: bad argument");
    const int64_t pk = elem_off[count] + 3;
    const int64_t need = framed ? xhe_zstd_raw_frame_size(pk) : pk;
    *out_len = need;
    if (need > cap) return xhe_fail(XHE_EOVERFLOW, "xhe_wire_finish: output buffer smaller than the payload");
    xhe::wire::write_foot(elem_off[count], xhe::wire::Sink{out, framed ? kZstdBlock : 0});
    if (framed) write_frame_headers(out, pk);
    return XHE_OK;
  });
}

int xhe_wire_decode(const uint8_t* data, int64_t len, int n2w, uint32_t* ct, int32_t* exps, int64_t cap_count,
                    int64_t* count, int64_t* shape, int* ndim) {
  return guarded([&]() -> int {
    if (!data || len <= 0 || n2w <= 0 || !count || !shape || !ndim || (cap_count > 0 && (!ct || !exps)))
      return xhe_fail(XHE_EINVAL, "xhe_wire_decode: bad argument");
    int64_t n = xhe::wire::decode(data, len, n2w, ct, exps, cap_count, shape, ndim);
    *count = n;
    if (n > cap_count) return xhe_fail(XHE_EOVERFLOW, "xhe_wire_decode: output buffers too small");
    return XHE_OK;
  });
}

const char* xhe_last_error(void) { return g_err.c_str(); }
const char* xhe_version(void) { return "xhe 0.2 gfx950"; }

}  // extern "C"
