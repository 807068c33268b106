// Issue rate of the VALU operations the strict UTF-8 check is built from, on
// a full chip: every SIMD holds `waves` waves, each running 8 independent
// chains of one operation.  Prints SIMD cycles per wave64 instruction (2.0 =
// full rate on a SIMD-32), counted by the shader clock itself (s_memtime
// around each wave's loop; the 100 MHz s_memrealtime beside it gives the
// clock), and the same from the event time at --ghz.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate
// run:   tools/valu_rate [waves_per_simd=8] [ghz=2.4]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define OP_LOOP(NAME, ASM)                                                                \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned long long* cyc, unsigned iters, unsigned s) { \
    unsigned a0 = threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u,      \
             a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;                                  \
    const unsigned b = s * 0x01010101u, c = s ^ 0x03020100u;                               \
    const unsigned long long t0 = clock64(), r0 = wall_clock64();                          \
    for (unsigned i = 0; i < iters; ++i) {                                                 \
      asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                       \
      asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c));                                       \
      asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c));                                       \
      asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c));                                       \
      asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c));                                       \
      asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c));                                       \
      asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c));                                       \
      asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c));                                       \
    }                                                                                      \
    const unsigned long long t1 = clock64(), r1 = wall_clock64();                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;    \
    if ((threadIdx.x & 63u) == 0) {                                                        \
      const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;                     \
      cyc[2 * w] = t1 - t0;                                                                \
      cyc[2 * w + 1] = r1 - r0;                                                            \
    }                                                                                      \
  }

#define OP_LOOP64(NAME, ASM)                                                              \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned long long* cyc, unsigned iters, unsigned s) { \
    unsigned long long a0 = threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, \
                       a5 = a0 * 13u, a6 = a0 * 17u, a7 = a0 * 19u;                        \
    const unsigned long long b = s * 0x0101010101010101ull;                                \
    const unsigned long long t0 = clock64(), r0 = wall_clock64();                          \
    for (unsigned i = 0; i < iters; ++i) {                                                 \
      asm volatile(ASM : "+v"(a0) : "v"(b));                                               \
      asm volatile(ASM : "+v"(a1) : "v"(b));                                               \
      asm volatile(ASM : "+v"(a2) : "v"(b));                                               \
      asm volatile(ASM : "+v"(a3) : "v"(b));                                               \
      asm volatile(ASM : "+v"(a4) : "v"(b));                                               \
      asm volatile(ASM : "+v"(a5) : "v"(b));                                               \
      asm volatile(ASM : "+v"(a6) : "v"(b));                                               \
      asm volatile(ASM : "+v"(a7) : "v"(b));                                               \
    }                                                                                      \
    const unsigned long long t1 = clock64(), r1 = wall_clock64();                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
    if ((threadIdx.x & 63u) == 0) {                                                        \
      const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;                     \
      cyc[2 * w] = t1 - t0;                                                                \
      cyc[2 * w + 1] = r1 - r0;                                                            \
    }                                                                                      \
  }

OP_LOOP(k_and, "v_and_b32 %0, %0, %1")
OP_LOOP(k_lshl, "v_lshlrev_b32 %0, 3, %0")
OP_LOOP(k_perm, "v_perm_b32 %0, %0, %1, %2")
OP_LOOP(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 3")
OP_LOOP(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe4")
OP_LOOP(k_or3, "v_or3_b32 %0, %0, %1, %2")
OP_LOOP(k_add, "v_add_u32 %0, %0, %1")
OP_LOOP(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
OP_LOOP(k_and64, "v_and_b32_e64 %0, %0, %1")
OP_LOOP(k_lshl64, "v_lshlrev_b32_e64 %0, 3, %0")
OP_LOOP(k_lshr, "v_lshrrev_b32 %0, 3, %0")
OP_LOOP(k_lshlor, "v_lshl_or_b32 %0, %0, 4, %1")
OP_LOOP(k_andor, "v_and_or_b32 %0, %0, %1, %2")
OP_LOOP(k_xor, "v_xor_b32 %0, %0, %1")
OP_LOOP(k_bitop3b, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x6a")
OP_LOOP(k_alignbit, "v_alignbit_b32 %0, %0, %1, 4")
OP_LOOP(k_perm2, "v_perm_b32 %0, %1, %0, %2")
OP_LOOP64(k_lshl64b, "v_lshlrev_b64 %0, 4, %0")
OP_LOOP64(k_lshr64b, "v_lshrrev_b64 %0, 4, %0")
OP_LOOP64(k_lshladd64, "v_lshl_add_u64 %0, %0, 4, %1")
OP_LOOP(k_pklshl, "v_pk_lshlrev_b16 %0, 4, %0")
OP_LOOP(k_pkadd, "v_pk_add_u16 %0, %0, %1")
OP_LOOP(k_bfe, "v_bfe_u32 %0, %0, 4, 3")

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 8;
  const double ghz = argc > 2 ? atof(argv[2]) : 2.4;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int cus = p.multiProcessorCount;
  const unsigned blocks = (unsigned)(cus * waves);  // 4 waves a block: `waves` per SIMD
  const unsigned iters = 4096;
  unsigned* out = nullptr;
  unsigned long long* cyc = nullptr;
  const size_t nw = (size_t)blocks * 4;
  if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
  if (hipMalloc(&cyc, nw * 16) != hipSuccess) return 1;
  unsigned long long* h = (unsigned long long*)malloc(nw * 16);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct K {
    const char* name;
    void (*fn)(unsigned*, unsigned long long*, unsigned, unsigned);
  } ks[] = {{"v_and_b32", k_and},         {"v_lshlrev_b32", k_lshl}, {"v_perm_b32", k_perm},
            {"v_alignbyte_b32", k_alignbyte}, {"v_bitop3_b32", k_bitop3}, {"v_or3_b32", k_or3},
            {"v_add_u32", k_add},         {"v_bfi_b32", k_bfi},   {"v_and_b32_e64", k_and64},
            {"v_lshlrev_b32_e64", k_lshl64}, {"v_lshrrev_b32", k_lshr}, {"v_lshl_or_b32", k_lshlor},
            {"v_and_or_b32", k_andor},    {"v_xor_b32", k_xor},   {"v_bitop3_b32_0x6a", k_bitop3b},
            {"v_alignbit_b32", k_alignbit}, {"v_perm_b32_b", k_perm2}, {"v_lshlrev_b64", k_lshl64b},
            {"v_lshrrev_b64", k_lshr64b}, {"v_lshl_add_u64", k_lshladd64}, {"v_pk_lshlrev_b16", k_pklshl},
            {"v_pk_add_u16", k_pkadd},    {"v_bfe_u32", k_bfe}};
  printf("{\"cus\": %d, \"waves_per_simd\": %d, \"ghz_assumed\": %.3f, \"simd_cycles_per_wave_instr\": {", cus, waves,
         ghz);
  for (size_t k = 0; k < sizeof ks / sizeof ks[0]; ++k) {
    hipLaunchKernelGGL(ks[k].fn, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1u);  // warm
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ks[k].fn, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1u);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per SIMD: waves per SIMD x iters x 8
    const double per_simd = (double)waves * iters * 8.0 * 5.0;
    const double ev = ms * 1e-3 * ghz * 1e9 / per_simd;
    (void)hipMemcpy(h, cyc, nw * 16, hipMemcpyDeviceToHost);
    double sc = 0, sr = 0;
    for (size_t w = 0; w < nw; ++w) {
      sc += (double)h[2 * w];
      sr += (double)h[2 * w + 1];
    }
    // a wave's loop: iters x 8 of its own instructions, `waves` waves sharing the SIMD
    const double per_wave = sc / nw / (iters * 8.0);
    printf("%s\"%s\": {\"clk_per_instr_per_wave\": %.3f, \"simd_clk_per_instr\": %.3f, \"ghz\": %.3f, "
           "\"event_at_ghz_arg\": %.3f}",
           k ? ", " : "", ks[k].name, per_wave, per_wave / waves, sc / sr * 0.1, ev);  // s_memrealtime ticks at 100 MHz
  }
  printf("}}\n");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
