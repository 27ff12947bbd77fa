// membench6.hip — phased-write probes for the RS(30,3) pass (measurement tool,
// not product code).
//
// membench5 showed that the first parity write stream costs far more than its
// bytes (30 reads + 1 write: +0.13 ms for 134 MB, ~1 TB/s marginal), while a
// sequential copy with 50% writes runs at 6.3 TB/s.  These probes buffer a
// workgroup's parity tiles in LDS and write them as one contiguous burst per
// phase (T tiles -> T x 8 KiB contiguous per output shard), optionally with a
// grid-wide barrier so every CU writes in the same window (SYNC=1).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/membench6.hip -o tools/membench6
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));           \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Args {
  uint64_t in[120];  // K * B shard addresses
  uint64_t out[12];  // 3 * B
  uint32_t K, B;
  uint32_t tiles_per_block;
  uint32_t total_tiles;
};

__device__ __forceinline__ void gload2(u32x4 &L, u32x4 &H, uint64_t base, uint32_t voff) {
  asm volatile("global_load_dwordx4 %0, %2, %3\n\tglobal_load_dwordx4 %1, %2, %3 offset:32"
               : "=&v"(L), "=&v"(H) : "v"(voff), "s"(base) : "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait(u32x4 &L, u32x4 &H) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(L), "+v"(H) : "n"(N) : "memory");
}

template <int SPOL>
__device__ __forceinline__ void gstore(uint64_t base, uint32_t voff, const u32x4 &v) {
  if constexpr (SPOL == 0)
    asm volatile("global_store_dwordx4 %0, %1, %2" ::"v"(voff), "v"(v), "s"(base) : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, %2 nt" ::"v"(voff), "v"(v), "s"(base) : "memory");
}

__device__ __forceinline__ uint32_t tile_voff(uint32_t tile, uint32_t thread) {
  const uint64_t hc = uint64_t(tile) * 256 + thread;
  return uint32_t((hc >> 1) * 64 + (hc & 1) * 16);
}

// The product kernel's read ring over K inputs for one tile; XOR-accumulate.
// The product kernel's read ring over K inputs for one tile; XOR-accumulate.
__device__ __forceinline__ void read_tile(const Args &a, uint32_t t, uint32_t wave, uint32_t lane256,
                                          u32x4 &accL, u32x4 &accH) {
  const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
  const uint32_t voff = tile_voff(tile, lane256);
  const uint64_t *in = a.in + b * a.K;
  const uint32_t K = a.K;
  const uint32_t rot = (tile * 4 + wave) % K;
  auto idx = [&](uint32_t x) -> uint32_t {
    if (x >= K) x = K - 1;
    const uint32_t y = rot + x;
    return y >= K ? y - K : y;
  };
  accL = u32x4{0, 0, 0, 0};
  accH = u32x4{0, 0, 0, 0};
  u32x4 LA, HA, LB, HB, LC, HC, LD, HD;
  gload2(LA, HA, in[idx(0)], voff);
  gload2(LB, HB, in[idx(1)], voff);
  gload2(LC, HC, in[idx(2)], voff);
  for (uint32_t i = 0;; i += 4) {
    gload2(LD, HD, in[idx(i + 3)], voff);
    vm_wait<6>(LA, HA);
    accL ^= LA; accH ^= HA;
    gload2(LA, HA, in[idx(i + 4)], voff);
    vm_wait<6>(LB, HB);
    accL ^= LB; accH ^= HB;
    if (i + 2 >= K) break;
    gload2(LB, HB, in[idx(i + 5)], voff);
    vm_wait<6>(LC, HC);
    accL ^= LC; accH ^= HC;
    gload2(LC, HC, in[idx(i + 6)], voff);
    vm_wait<6>(LD, HD);
    accL ^= LD; accH ^= HD;
    if (i + 4 >= K) break;
  }
  vm_wait<0>(LA, HA);
}


__device__ __forceinline__ uint32_t spin_until(uint32_t *cnt, uint32_t target) {
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t v;
  while ((v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) return 1;  // 100 ms: give up
  }
  return 0;
}

// NW compute waves per workgroup = NW/4 tile groups; T tiles per phase
// (T % (NW/4) == 0); LDS image [tile][out][8 KiB] in shard byte order.
// OM: burst order output-major (each output's T x 8 KiB run stored in one
// sweep).  WW: extra writer waves (one per SIMD) that own the burst, so
// compute waves never wait on store acknowledgements (vmcnt counts stores).
template <int NW, int T, int SYNC, int SPOL, int OM = 0, int WW = 0>
__global__ __launch_bounds__((NW + WW) * 64) void phased(const Args a, uint32_t *cnt) {
  extern __shared__ u32x4 img[];  // T * 3 * 512 x 16 B
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t G = gridDim.x, total = a.total_tiles;
  const uint32_t per_phase = G * T;
  const uint32_t n_phase = (total + per_phase - 1) / per_phase;
  auto burst = [&](uint32_t base, uint32_t first, uint32_t stride) {
    const uint32_t n16 = T * 3 * 512;
    for (uint32_t e = first; e < n16; e += stride) {
      uint32_t j, o;
      if (OM) { o = e / (T * 512); j = (e / 512) % T; }
      else { j = e / 1536; o = (e / 512) % 3; }
      const uint32_t r = e % 512;
      const uint32_t t = base + j;
      if (t >= total) continue;
      const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
      const uint64_t dst = a.out[b * 3 + o] + uint64_t(tile) * 8192 + r * 16;
      const u32x4 v = img[(j * 3 + o) * 512 + r];
      if (SPOL) __builtin_nontemporal_store(v, (u32x4 *)dst);
      else *(u32x4 *)dst = v;
    }
  };
  if (WW && wave >= NW) {
    for (uint32_t p = 0; p < n_phase; ++p) {
      asm volatile("s_barrier" ::: "memory");  // A(p): image full
      burst(p * per_phase + blockIdx.x * T, threadIdx.x - NW * 64, WW * 64);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B(p): image read
    }
    return;
  }
  const uint32_t grp = wave >> 2, w4 = wave & 3, l256 = threadIdx.x & 255;
  for (uint32_t p = 0; p < n_phase; ++p) {
    const uint32_t base = p * per_phase + blockIdx.x * T;
    for (uint32_t jj = 0; jj < T / (NW / 4); ++jj) {
      const uint32_t j = grp + jj * (NW / 4);
      const uint32_t t = base + j;
      const bool valid = t < total;  // wave-uniform
      u32x4 accL = {0, 0, 0, 0}, accH = {0, 0, 0, 0};
      if (valid) read_tile(a, t, w4, l256, accL, accH);
      if (WW && p > 0 && jj == 0) asm volatile("s_barrier" ::: "memory");  // B(p-1), every wave
      if (!valid) continue;
      const uint32_t hc = l256;
      const uint32_t rel = ((hc >> 1) * 64 + (hc & 1) * 16) >> 4;  // in 16-B units
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        u32x4 *d = img + (j * 3 + o) * 512 + rel;
        d[0] = accL + u32x4{uint32_t(o), 0, 0, 0};
        d[2] = accH + u32x4{uint32_t(o), 0, 0, 0};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // A(p)
    if (WW) continue;
    if (SYNC) {
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        spin_until(cnt, G * (p + 1));
      }
      asm volatile("s_barrier" ::: "memory");
    }
    burst(base, threadIdx.x, NW * 64);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (WW && n_phase > 0) asm volatile("s_barrier" ::: "memory");  // B(last)
}

template <int WRITES>
__global__ __launch_bounds__(256) void base_probe(const Args a) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t t = blockIdx.x;
  u32x4 accL, accH;
  read_tile(a, t, wave, threadIdx.x, accL, accH);
  const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
  const uint32_t voff = tile_voff(tile, threadIdx.x);
  if constexpr (WRITES) {
    const uint64_t *out = a.out + b * 3;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      gstore<1>(out[o], voff, accL + u32x4{uint32_t(o), 0, 0, 0});
      gstore<1>(out[o], voff + 32, accH + u32x4{uint32_t(o), 0, 0, 0});
    }
  } else {
    if (accL.x == 0x12345678u && accH.y == 0x9abcdef0u) gstore<0>(a.out[0], voff, accL);
  }
}

int main(int argc, char **argv) {
  const uint32_t K = 30, B = 4;
  const uint64_t S = 32ull << 20;
  uint8_t *data, *par;
  uint32_t *cnt;
  CHECK(hipMalloc(&data, S * K * B));
  CHECK(hipMalloc(&par, S * 3 * B));
  CHECK(hipMalloc(&cnt, 4096));
  CHECK(hipMemset(data, 0x5a, S * K * B));
  CHECK(hipMemset(par, 0, S * 3 * B));
  const uint32_t tpb = uint32_t(S / 8192);
  Args a{};
  for (uint32_t i = 0; i < K * B; ++i) a.in[i] = uint64_t(data) + S * i;
  for (uint32_t i = 0; i < 3 * B; ++i) a.out[i] = uint64_t(par) + S * i;
  a.K = K;
  a.B = B;
  a.tiles_per_block = tpb;
  a.total_tiles = tpb * B;
  const double rs_bytes = double(S) * (K + 3) * B;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const uint32_t total = tpb * B;
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  {
    for (int i = 0; i < 600; ++i) hipLaunchKernelGGL((base_probe<1>), dim3(total), dim3(256), 0, 0, a);
    CHECK(hipDeviceSynchronize());
    printf("{\"settle\": \"ok\", \"cus\": %d}\n", ncu);
    fflush(stdout);
  }
  auto time = [&](const char *name, auto launch, double nbytes) {
    fprintf(stderr, "start %s\n", name);
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipDeviceSynchronize());
    const int iters = 20;
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      best = ms < best ? ms : best;
    }
    printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, best, nbytes / best / 1e6);
    fflush(stdout);
  };
  time("base", [&] { hipLaunchKernelGGL((base_probe<1>), dim3(total), dim3(256), 0, 0, a); }, rs_bytes);
  auto run = [&](auto kfn, int nw, int T, int sync, int sp, int om, int ww) {
    const size_t lds = size_t(T) * 3 * 8192;
    int per = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, (nw + ww) * 64, lds));
    if (per < 1) { printf("{\"skip\": %d}\n", T); return; }
    const uint32_t G = uint32_t(per * ncu);
    char name[96];
    snprintf(name, sizeof name, "ph_nw%d_t%d_sync%d_s%d_om%d_ww%d_per%d", nw, T, sync, sp, om, ww, per);
    time(name, [&] {
      hipMemsetAsync(cnt, 0, 4096, 0);
      hipLaunchKernelGGL(kfn, dim3(G), dim3((nw + ww) * 64), lds, 0, a, cnt);
    }, rs_bytes);
  };
  run(phased<8, 6, 0, 1>, 8, 6, 0, 1, 0, 0);
  run(phased<8, 6, 0, 1, 1>, 8, 6, 0, 1, 1, 0);
  run(phased<4, 6, 0, 1, 1>, 4, 6, 0, 1, 1, 0);
  run(phased<4, 6, 0, 1, 0, 4>, 4, 6, 0, 1, 0, 4);
  run(phased<4, 6, 0, 1, 1, 4>, 4, 6, 0, 1, 1, 4);
  run(phased<8, 6, 0, 1, 1, 4>, 8, 6, 0, 1, 1, 4);
  run(phased<12, 6, 0, 1, 1, 4>, 12, 6, 0, 1, 1, 4);
  run(phased<8, 4, 0, 1, 1, 4>, 8, 4, 0, 1, 1, 4);
  run(phased<4, 6, 0, 0, 1, 4>, 4, 6, 0, 0, 1, 4);
  run(phased<4, 3, 0, 1, 1, 4>, 4, 3, 0, 1, 1, 4);
  time("base_again", [&] { hipLaunchKernelGGL((base_probe<1>), dim3(total), dim3(256), 0, 0, a); }, rs_bytes);
  return 0;
}
