// simd_probe.hip — where do a 256-thread workgroup's four waves run?
// Each wave records its HW_ID (SIMD, CU, SE) and XCC_ID; the host reports
// how often wave w of a workgroup sits on SIMD s, and how often the
// workgroups resident on one CU put wave 0 on the same SIMD.  It decides
// whether the device BLAKE3's narrow tree levels (done by wave 0 alone)
// pile onto one SIMD per CU.  Measurement only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ __launch_bounds__(256) void probe(uint32_t *out, uint32_t spin) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // keep the workgroup resident a while so many are co-resident per CU
  uint32_t x = threadIdx.x;
  for (uint32_t i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
  if ((threadIdx.x & 63) == 0) {
    out[3 * (blockIdx.x * 4 + threadIdx.x / 64)] = hw;
    out[3 * (blockIdx.x * 4 + threadIdx.x / 64) + 1] = xcc;
    out[3 * (blockIdx.x * 4 + threadIdx.x / 64) + 2] = x;
  }
}

int main(int argc, char **argv) {
  const uint32_t nwg = argc > 1 ? atoi(argv[1]) : 16384;
  const uint32_t spin = argc > 2 ? atoi(argv[2]) : 20000;
  uint32_t *d;
  if (hipMalloc(&d, size_t(nwg) * 4 * 3 * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), 0, 0, d, spin);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<uint32_t> h(size_t(nwg) * 4 * 3);
  if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  long per[4][4] = {};  // [wave][simd]
  long spread[5] = {};  // distinct SIMDs used by one workgroup's 4 waves
  std::map<uint64_t, std::vector<uint32_t>> wave0;  // CU key -> wave-0 SIMDs over time
  for (uint32_t b = 0; b < nwg; ++b) {
    uint32_t mask = 0;
    for (uint32_t w = 0; w < 4; ++w) {
      const uint32_t hw = h[3 * (b * 4 + w)], xcc = h[3 * (b * 4 + w) + 1] & 0xf;
      const uint32_t simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1,
                     se = (hw >> 13) & 7;
      per[w][simd]++;
      mask |= 1u << simd;
      if (w == 0) wave0[(uint64_t(xcc) << 16) | (se << 8) | (sh << 4) | cu].push_back(simd);
    }
    spread[__builtin_popcount(mask)]++;
  }
  printf("{\"workgroups\": %u, \"wave_simd\": [", nwg);
  for (int w = 0; w < 4; ++w)
    printf("%s[%ld, %ld, %ld, %ld]", w ? ", " : "", per[w][0], per[w][1], per[w][2], per[w][3]);
  printf("], \"distinct_simds_per_wg\": [%ld, %ld, %ld, %ld], \"cus\": %zu",
         spread[1], spread[2], spread[3], spread[4], wave0.size());
  long same = 0, total = 0;
  for (auto &kv : wave0) {
    long c[4] = {};
    for (uint32_t s : kv.second) c[s]++;
    long mx = 0;
    for (long v : c) mx = v > mx ? v : mx;
    same += mx;
    total += long(kv.second.size());
  }
  printf(", \"wave0_on_modal_simd_frac\": %.3f}\n", total ? double(same) / total : 0.0);
  return 0;
}
