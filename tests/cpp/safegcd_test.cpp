// Host build of csrc/safegcd.h (the device Fp inversion) for tests/test_safegcd.py: reads
// canonical values as 12 little-endian u32 words per line (hex) on stdin, writes their inverses
// mod p the same way, plus the number of 30-divstep batches each one took.
#include <stdio.h>

#include "../../bellman-mpc_amd/csrc/safegcd.h"

static int batches_of(const int32_t* x0) {
  // the same loop as sg_inverse, counting batches (termination bound check)
  int32_t d[bh::SG_NL] = {0}, e[bh::SG_NL] = {0}, f[bh::SG_NL], g[bh::SG_NL];
  for (int i = 0; i < bh::SG_NL; ++i) {
    f[i] = FpInvCfg::M30[i];
    g[i] = x0[i];
  }
  e[0] = 1;
  int32_t zeta = -1;
  for (int it = 0; it < 64; ++it) {
    bh::SgT t;
    zeta = bh::sg_divsteps30(zeta, (uint32_t)f[0], (uint32_t)g[0], t);
    bh::sg_update_de(d, e, t);
    bh::sg_update_fg(f, g, t);
    int32_t nz = 0;
    for (int i = 0; i < bh::SG_NL; ++i) nz |= g[i];
    if (nz == 0) return it + 1;
  }
  return -1;
}

int main() {
  uint32_t w[12];
  while (true) {
    for (int k = 0; k < 12; ++k)
      if (scanf("%x", &w[k]) != 1) return 0;
    // 12 x 32 -> 14 x 29
    uint32_t a[14];
    unsigned __int128 acc = 0;
    int bits = 0, j = 0;
    for (int k = 0; k < 12; ++k) {
      acc |= (unsigned __int128)w[k] << bits;
      bits += 32;
      while (bits >= 29 && j < 14) {
        a[j++] = (uint32_t)(acc & 0x1fffffff);
        acc >>= 29;
        bits -= 29;
      }
    }
    while (j < 14) {
      a[j++] = (uint32_t)(acc & 0x1fffffff);
      acc >>= 29;
    }
    int32_t s[bh::SG_NL];
    bh::sg_from29(a, s);
    const int nb = batches_of(s);
    bh::sg_inverse(s);
    uint32_t b[14];
    bh::sg_to29(s, b);
    // 14 x 29 -> 12 x 32
    acc = 0;
    bits = 0;
    j = 0;
    uint32_t o[12];
    for (int k = 0; k < 14; ++k) {
      acc |= (unsigned __int128)b[k] << bits;
      bits += 29;
      while (bits >= 32 && j < 12) {
        o[j++] = (uint32_t)acc;
        acc >>= 32;
        bits -= 32;
      }
    }
    while (j < 12) {
      o[j++] = (uint32_t)acc;
      acc >>= 32;
    }
    for (int k = 0; k < 12; ++k) printf("%08x ", o[k]);
    printf("%d\n", nb);
  }
}
