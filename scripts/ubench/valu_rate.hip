// Microbenchmark: VALU issue cost per instruction type (many waves, independent chains).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP, int C>
__global__ __launch_bounds__(256) void valu(int steps, uint32_t seed, uint32_t* out) {
  uint32_t x[C], y[C];
#pragma unroll
  for (int c = 0; c < C; ++c) { x[c] = threadIdx.x * 7 + c + seed; y[c] = x[c] * 13 + 1; }
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if (OP == 0) x[c] = x[c] + y[c];
        if (OP == 1) x[c] = __builtin_amdgcn_alignbit(x[c], y[c], x[c]);
        if (OP == 2) x[c] = (x[c] >> (y[c] & 31)) ^ y[c];  // 2 ops-ish
        if (OP == 3) x[c] = __builtin_amdgcn_ubfe(x[c], y[c] & 31, 5) + y[c];
        if (OP == 4) x[c] = __builtin_amdgcn_perm(x[c], y[c], 0x05010400u + k);
        if (OP == 5) x[c] = __builtin_amdgcn_alignbyte(x[c], y[c], x[c]);
        if (OP == 6) x[c] = x[c] * y[c];
        if (OP == 7) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(x[c]) : "v"(y[c]));
        if (OP == 8) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x[c]) : "v"(y[c]));
        if (OP == 9) { uint64_t w = ((uint64_t)x[c] << 32) | y[c]; asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(w) : "v"(x[c])); x[c] = (uint32_t)w; }
        if (OP == 10) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x[c]) : "v"(y[c]));
        if (OP == 11) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y[c]));
        if (OP == 12) asm volatile("v_bfe_u32 %0, %0, 8, 5" : "+v"(x[c]));
        if (OP == 13) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(x[c]));
        if (OP == 14) asm volatile("v_alignbit_b32 %0, %0, %1, %0" : "+v"(x[c]) : "v"(y[c]));
        if (OP == 15) asm volatile("v_cmp_gt_i32 vcc, %1, %0\n v_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(x[c]) : "v"(y[c]) : "vcc");
      }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) acc ^= x[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int OP, int C>
void run(const char* name, int wg, int ncu, uint32_t* d) {
  const int steps = 2048;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL((valu<OP, C>), dim3(wg * ncu), dim3(256), 0, 0, 4, 1u, d);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((valu<OP, C>), dim3(wg * ncu), dim3(256), 0, 0, steps, 1u, d);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double winstr_per_simd = double(wg) * 16.0 * C * steps;  // wg waves per SIMD
  printf("%-10s C=%d waves/simd=%d: %.3f ms  %.2f cyc/wave-instr/SIMD (at 2.4GHz)\n", name, C, wg, ms,
         ms * 1e-3 * 2.4e9 / winstr_per_simd);
}

int main() {
  int ncu;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* d;
  (void)hipMalloc(&d, 8 * 256 * ncu * 4);
  for (int wg : {1, 4, 8}) {
    run<0, 4>("add", wg, ncu, d);
    run<1, 4>("alignbit", wg, ncu, d);
    run<2, 4>("shr+xor+and", wg, ncu, d);
    run<3, 4>("bfe+add", wg, ncu, d);
    run<4, 4>("perm", wg, ncu, d);
    run<5, 4>("alignbyte", wg, ncu, d);
    run<6, 4>("mul_lo", wg, ncu, d);
    run<7, 4>("sdwa_mov", wg, ncu, d);
    run<8, 4>("sdwa_add", wg, ncu, d);
    run<9, 4>("lshr_b64", wg, ncu, d);
    run<10, 4>("lshl_add", wg, ncu, d);
    run<11, 4>("add(asm)", wg, ncu, d);
    run<12, 4>("bfe(asm)", wg, ncu, d);
    run<13, 4>("lshr(asm)", wg, ncu, d);
    run<14, 4>("alignbit(asm)", wg, ncu, d);
    run<15, 4>("cmp+addc", wg, ncu, d);
  }
  return 0;
}
