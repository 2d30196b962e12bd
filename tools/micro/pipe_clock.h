// Per-phase cycles of a clocked LDS-DMA pipeline launch (csrc/gemm_pipe.h
// PIPE_CLK slots, -DOAC_PIPE_CLOCK builds): averaged over the launch's workgroups.
#pragma once
#include <algorithm>
#include <cstdio>
#include <vector>

static void print_pipe_clocks(int total_tiles) {
  const int n = total_tiles < 4096 ? total_tiles : 4096;
  std::vector<long long> c((size_t)n * 32);
  CK(hipMemcpyFromSymbol(c.data(), HIP_SYMBOL(oac::g_pipe_clock), c.size() * 8));
  long long t0 = c[0], tend = 0;
  for (int i = 0; i < n; ++i) { t0 = std::min(t0, c[i * 32]); tend = std::max(tend, c[i * 32 + 31]); }
  double st[32] = {0};
  int nst = 0;
  while (nst < 27 && c[2 + nst] > c[1]) ++nst;
  for (int i = 0; i < n; ++i) {
    const long long* r = &c[(size_t)i * 32];
    st[0] += r[1] - r[0];                 // task lookup -> pipe start
    st[1] += r[2] - r[1];                 // prologue issue -> stage 0 ready
    for (int k = 1; k < nst; ++k) st[1 + k] += r[2 + k] - r[1 + k];
    st[28] += r[29] - r[1 + nst];         // last stage compute
    st[29] += r[30] - r[29];              // epilogue
    st[30] += r[31] - r[30];              // continuation + 2nd epilogue
    st[31] += r[0] - t0;                  // start skew
  }
  printf("  clocks (cycles, avg over %d wgs, %d stages): start skew %.0f  lookup %.0f  prologue %.0f  stages",
         n, nst, st[31] / n, st[0] / n, st[1] / n);
  for (int k = 1; k < nst; ++k) printf(" %.0f", st[1 + k] / n);
  printf("  last %.0f  epilogue %.0f  cont %.0f | span %lld\n", st[28] / n, st[29] / n, st[30] / n, tend - t0);
}

