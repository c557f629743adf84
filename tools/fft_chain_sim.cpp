// fft_chain_sim.cpp — TEST INFRASTRUCTURE: a host model of the coarse
// kernel's chained transforms (aero-cli_amd/csrc/fft_chain.h) built on the
// same layout arithmetic (fft_layout.h).  It plays every lane of every wave:
// register stages with the kernel's twiddle indices and trivial-twiddle
// skips, the wave-local LDS transpose, v_permlane16_swap / v_permlane32_swap
// as the ISA defines them (odd rows of vdst <-> even rows of src; upper half
// of vdst <-> lower half of src) and the workgroup G exchange, then writes
// each value to its natural bin.  tests/test_fft_chain_sim.py checks the
// result against the oracle's JFFT (decode/jfft.cpp:114-212) chain
// forward -> boxcar -> inverse -> square -> forward, bit for bit up to the
// sign of exact zeros, so the index arithmetic is proven on the CPU before
// the kernel runs it.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../aero-cli_amd/csrc/fft_layout.h"

using namespace aero::fftl;

namespace {

struct C {
  double x, y;
};

template <int L>
struct Sim {
  static constexpr int T = 1 << (L - 4), N = 1 << L;
  std::vector<C> v = std::vector<C>((size_t)T * 16);
  std::vector<double> lds = std::vector<double>((size_t)N + N / 16);
  const C *tw = nullptr, *twi = nullptr;
  // the permuted copies the kernel reads its G-layout stages past the LDS
  // twiddles from (fft_layout.h twg_build)
  std::vector<C> twg = std::vector<C>((size_t)N), twgi = std::vector<C>((size_t)N);
  void set_tables(const C *f, const C *i) {
    tw = f;
    twi = i;
    twg_build<L>(reinterpret_cast<const double *>(f), reinterpret_cast<double *>(twg.data()));
    twg_build<L>(reinterpret_cast<const double *>(i), reinterpret_cast<double *>(twgi.data()));
  }

  C &at(int t, int i) { return v[(size_t)t * 16 + i]; }

  template <uint64_t LAY, int KIND, bool FIRST, int S, bool INV>
  void stage() {
    constexpr int rb = sb(LAY, S), n = 1 << S;
    static_assert(rb < 4, "stage bit in a register");
    constexpr bool thread_low = (thread_mask(LAY, L) & (n - 1)) != 0;
    const C *table = INV ? twi : tw;
    for (int t = 0; t < T; t++) {
      const int a = athr<L, KIND, FIRST>(t);
      for (int i = 0; i < 16; i++) {
        if (i & (1 << rb)) continue;
        const int il = i | (1 << rb);
        const int kr = areg(LAY, L, i) & (n - 1);
        C &xi = at(t, i), &xl = at(t, il);
        double yr, yi;
        if (!thread_low && kr == 0) {  // TW[n - 1] = (1, +-0): the kernel skips the product
          yr = xl.x;
          yi = xl.y;
        } else {
          constexpr bool perm = KIND == K_G && n > (L >= 14 ? 512 : 256);  // TwLds<L>::N
          const C w = perm ? (INV ? twgi : twg)[(size_t)(twg_base<L>(S) + twg_row<L>(S, i)) * T + t]
                           : table[n - 1 + ((a & (n - 1)) | kr)];
          yr = w.x * xl.x - w.y * xl.y;
          yi = w.x * xl.y + w.y * xl.x;
        }
        xl.x = xi.x - yr;
        xl.y = xi.y - yi;
        xi.x = xi.x + yr;
        xi.y = xi.y + yi;
      }
    }
  }

  void wl() {  // per wave, re then im, through the wave's LDS region
    for (int part = 0; part < 2; part++)
      for (int w = 0; w < T / 64; w++) {
        double *base = lds.data() + (size_t)w * WL_REGION;
        for (int l = 0; l < 64; l++)
          for (int i = 0; i < 16; i++) base[wl_w(l, i)] = part ? at(w * 64 + l, i).y : at(w * 64 + l, i).x;
        for (int l = 0; l < 64; l++)
          for (int i = 0; i < 16; i++) (part ? at(w * 64 + l, i).y : at(w * 64 + l, i).x) = base[wl_r(l, i)];
      }
  }

  void perm() {
    for (int w = 0; w < T / 64; w++) {
      for (int i = 0; i < 16; i++) {
        if (!(i & 4)) {  // v_permlane16_swap(vdst = x[i], src = x[i | 4]): rows 1, 3 of vdst <-> rows 0, 2 of src
          for (int m = 0; m < 16; m++) {
            std::swap(at(w * 64 + 16 + m, i), at(w * 64 + m, i | 4));
            std::swap(at(w * 64 + 48 + m, i), at(w * 64 + 32 + m, i | 4));
          }
        }
      }
      for (int i = 0; i < 16; i++) {
        if (!(i & 8)) {  // v_permlane32_swap(vdst = x[i], src = x[i | 8]): lanes 32-63 of vdst <-> 0-31 of src
          for (int m = 0; m < 32; m++) std::swap(at(w * 64 + 32 + m, i), at(w * 64 + m, i | 8));
        }
      }
    }
  }

  template <bool FIRST>
  void gx() {
    constexpr uint64_t P = lay_perm<L>(FIRST), G = lay_g<L>();
    for (int part = 0; part < 2; part++) {
      for (int t = 0; t < T; t++)
        for (int i = 0; i < 16; i++)
          lds[gidx(athr<L, K_PERM, FIRST>(t) | areg(P, L, i))] = part ? at(t, i).y : at(t, i).x;
      for (int t = 0; t < T; t++)
        for (int i = 0; i < 16; i++)
          (part ? at(t, i).y : at(t, i).x) = lds[gidx(athr<L, K_G, false>(t) | areg(G, L, i))];
    }
  }

  template <bool FIRST, bool INV>
  void fft() {
    constexpr uint64_t S0 = lay_start<L>(FIRST), W = lay_wl<L>(FIRST), P = lay_perm<L>(FIRST), G = lay_g<L>();
    stage<S0, K_START, FIRST, 0, INV>();
    stage<S0, K_START, FIRST, 1, INV>();
    stage<S0, K_START, FIRST, 2, INV>();
    stage<S0, K_START, FIRST, 3, INV>();
    wl();
    stage<W, K_WL, FIRST, 4, INV>();
    stage<W, K_WL, FIRST, 5, INV>();
    stage<W, K_WL, FIRST, 6, INV>();
    stage<W, K_WL, FIRST, 7, INV>();
    perm();
    stage<P, K_PERM, FIRST, 8, INV>();
    stage<P, K_PERM, FIRST, 9, INV>();
    gx<FIRST>();
    stage<G, K_G, false, 10, INV>();
    stage<G, K_G, false, 11, INV>();
    stage<G, K_G, false, 12, INV>();
    if (L == 14) stage<G, K_G, false, (L == 14 ? 13 : 12), INV>();
  }

  int bin(int t, int i) const { return athr<L, K_G, false>(t) | areg(lay_g<L>(), L, i); }

  void run(const C *in, int start, int stop, C *out) {
    for (int t = 0; t < T; t++)  // START of the first transform: a = i | t << 4, sample bitrev(a)
      for (int i = 0; i < 16; i++) at(t, i) = in[brev32((uint32_t)(i | (t << 4))) >> (32 - L)];
    fft<true, false>();
    for (int t = 0; t < T; t++)
      for (int i = 0; i < 16; i++) {
        const int k = bin(t, i);
        if (k >= start && k <= stop) at(t, i) = C{0.0, 0.0};
      }
    fft<false, true>();
    for (int t = 0; t < T; t++)
      for (int i = 0; i < 16; i++) {
        C &z = at(t, i);
        const double r = z.x * z.x - z.y * z.y, im = 2.0 * (z.x * z.y);
        z = C{r, im};
      }
    fft<false, false>();
    for (int t = 0; t < T; t++)
      for (int i = 0; i < 16; i++) out[bin(t, i)] = at(t, i);
  }
};

}  // namespace

extern "C" int fft_chain_sim(int L, const double *tw, const double *twi, const double *in, int start, int stop,
                             double *out) {
  if (L == 14) {
    Sim<14> s;
    s.set_tables(reinterpret_cast<const C *>(tw), reinterpret_cast<const C *>(twi));
    s.run(reinterpret_cast<const C *>(in), start, stop, reinterpret_cast<C *>(out));
    return 0;
  }
  if (L == 13) {
    Sim<13> s;
    s.set_tables(reinterpret_cast<const C *>(tw), reinterpret_cast<const C *>(twi));
    s.run(reinterpret_cast<const C *>(in), start, stop, reinterpret_cast<C *>(out));
    return 0;
  }
  return -1;
}
