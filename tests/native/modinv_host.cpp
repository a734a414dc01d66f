// CPU check of hostbn.hpp's modinv_words (host inverse at the root of the
// device batch inversion). Reads lines "nwords x_hex m_hex", prints the
// inverse as hex or "none".
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>
#include "../../xfl_amd/csrc/hostbn.hpp"

static void from_hex(const std::string& h, uint32_t* w, int nw) {
  std::memset(w, 0, nw * 4);
  int bit = 0;
  for (int i = (int)h.size() - 1; i >= 0 && bit < 32 * nw; --i, bit += 4) {
    char c = h[i];
    uint32_t v = (c >= '0' && c <= '9') ? c - '0' : (c | 32) - 'a' + 10;
    w[bit / 32] |= v << (bit % 32);
  }
}

int main() {
  int nw;
  std::string xs, ms;
  while (std::cin >> nw >> xs >> ms) {
    std::vector<uint32_t> x(nw), m(nw), y(nw);
    from_hex(xs, x.data(), nw);
    from_hex(ms, m.data(), nw);
    if (!xhe::modinv_words(x.data(), m.data(), nw, y.data())) {
      std::printf("none\n");
      continue;
    }
    for (int i = nw - 1; i >= 0; --i) std::printf("%08x", y[i]);
    std::printf("\n");
  }
  std::fprintf(stderr, "fallbacks %d\n", xhe::modinv_fallbacks().load());
  return 0;
}
