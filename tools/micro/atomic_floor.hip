// atomic_floor.hip -- the dQ traffic a fused key-major attention backward would add at
// cfg2 (B=8, H=16, T=4096, N=2 x hs=64 = 128 dQ columns), measured with no MFMA work:
// the floor under which such a kernel cannot go.
//
// One workgroup per (key block of BK keys, b*h); it walks the causal query steps of 32 rows
// from its key block to T.  Per step the workgroup's dQ contribution is a 32 x 128 fp32
// tile, already reduced over its BK keys: 4 waves each own 32 of the 128 columns and issue
// 16 no-return global_atomic_add_f32 per step (one 32x32 accumulator as it stands: lane l,
// register r -> row (r&3)+8(r>>2)+4(l>>5), column l&31 -- two 128-B segments per
// instruction, the full-rate shape of MI355X_MICROARCH.md 'Global float atomics').
// Mode "store" writes the same tiles with plain stores into per-key-block partial slabs
// instead (the atomic-free alternative, whose slabs a second pass then has to sum).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <bool ATOMIC>
__global__ __launch_bounds__(256) void dq_traffic(float* dq, int T, int BK, int nkb, long slab) {
  const int kb = blockIdx.x, bh = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = wave * 32 + (lane & 31);
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = 1e-3f * (r + 1);
  float* base = ATOMIC ? dq + (long)bh * T * 128 : dq + ((long)bh * nkb + kb) * slab;
  for (int q0 = kb * BK; q0 < T; q0 += 32) {
    float* tile = base + (long)(ATOMIC ? q0 : q0 - kb * BK) * 128 + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if constexpr (ATOMIC) __builtin_amdgcn_global_atomic_fadd_f32(tile + (long)row * 128, v[r]);
      else tile[(long)row * 128] = v[r];
    }
  }
}

int main(int argc, char** argv) {
  const int B = 8, H = 16, T = 4096;
  std::vector<int> bks = {128, 256, 512};
  printf("{\"what\": \"dQ fp32 traffic of a fused key-major backward at cfg2 (B=8 H=16 T=4096, 128 dQ columns), no MFMA\", \"rows\": [\n");
  bool first = true;
  for (int mode = 0; mode < 2; ++mode)
    for (int BK : bks) {
      const int nkb = T / BK;
      long steps = 0;
      for (int kb = 0; kb < nkb; ++kb) steps += (T - kb * BK) / 32;
      const double bytes = (double)steps * B * H * 32 * 128 * 4;
      const long slab = (long)T * 128;                 // per key block (upper bound)
      float* buf = nullptr;
      const size_t n = mode == 0 ? (size_t)B * H * T * 128 : (size_t)B * H * nkb * slab;
      if (hipMalloc(&buf, n * 4) != hipSuccess) { fprintf(stderr, "alloc failed\n"); return 1; }
      hipMemset(buf, 0, n * 4);
      dim3 grid(nkb, B * H);
      auto run = [&]() {
        if (mode == 0) hipLaunchKernelGGL(dq_traffic<true>, grid, dim3(256), 0, 0, buf, T, BK, nkb, slab);
        else hipLaunchKernelGGL(dq_traffic<false>, grid, dim3(256), 0, 0, buf, T, BK, nkb, slab);
      };
      for (int i = 0; i < 3; ++i) run();
      hipEvent_t a, b;
      hipEventCreate(&a); hipEventCreate(&b);
      const int reps = 10;
      hipEventRecord(a);
      for (int i = 0; i < reps; ++i) run();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      ms /= reps;
      printf("%s  {\"mode\": \"%s\", \"key_block\": %d, \"bytes\": %.0f, \"ms\": %.4f, \"TBps\": %.3f}", first ? "" : ",\n",
             mode == 0 ? "atomic_add_f32" : "plain_store_partials", BK, bytes, ms, bytes / ms / 1e9);
      first = false;
      hipFree(buf);
      hipEventDestroy(a); hipEventDestroy(b);
    }
  printf("\n]}\n");
  return 0;
}
