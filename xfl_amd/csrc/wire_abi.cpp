// Host-only part of the xhe C ABI (include/xhe.h): the wire codec entry
// points and the error channel. Compiled by the host compiler and linked into
// libxhe.so next to xhe.hip's object, so codec changes rebuild in seconds.
#include <stdint.h>

#include <algorithm>
#include <exception>
#include <string>
#include <thread>

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
int codec_threads() {
  unsigned hc = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(hc ? hc : 1u, 16u));
}
}  // namespace

int xhe_fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
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
