// membench3.hip — writer-wave probes for the RS(30,3) pass (measurement tool,
// not product code).
//
// Question: does the 3-stream parity write cost the product kernel ~18% of
// its time because compute waves wait for their stores to be acknowledged
// (store latency under a read-heavy load), rather than because of the bytes?
//
// Probes (XOR in place of the GF arithmetic; same lane layout and 4-buffer
// input ring as the product kernel; 4 x RS(30,3) blocks of 32 MiB shards):
//   base      one workgroup per 8 KiB tile, compute waves store their own outputs
//   ro        the same, reads only
//   ww<DB,SP> persistent grid, 4 compute waves + 1 writer wave per workgroup:
//             compute waves hand their outputs to LDS (DB = 1 or 2 buffers);
//             the writer wave stores them, so no compute wave ever waits on a
//             store.  SP: 0 plain, 1 nt stores.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/membench3.hip -o tools/membench3
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

// LDS barrier without a global-memory fence (a workgroup-scope __syncthreads
// may add vmcnt waits, which is exactly what the writer wave must avoid).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS slot layout: [buf][wave 4][out 3][half 2][lane 64] x 16 B = 24 KiB per buffer.
template <int DB, int SPOL>
__global__ __launch_bounds__(320) void ww_probe(const Args a) {
  extern __shared__ u32x4 slot[];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t G = gridDim.x;
  uint32_t j = 0;
  if (wave < 4) {
    for (uint32_t t = blockIdx.x; t < a.total_tiles; t += G, ++j) {
      u32x4 accL, accH;
      read_tile(a, t, wave, threadIdx.x, accL, accH);
      u32x4 *s = slot + (DB == 2 ? (j & 1) * 1536 : 0) + wave * 384 + lane;
      if (DB == 1) lds_barrier();  // A: writer has drained the buffer
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        s[(o * 2 + 0) * 64] = accL + u32x4{uint32_t(o), 0, 0, 0};
        s[(o * 2 + 1) * 64] = accH + u32x4{uint32_t(o), 0, 0, 0};
      }
      lds_barrier();  // B: buffer full
    }
  } else {
    for (uint32_t t = blockIdx.x; t < a.total_tiles; t += G, ++j) {
      if (DB == 1) lds_barrier();  // A
      lds_barrier();               // B
      const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
      const uint64_t *out = a.out + b * 3;
      const u32x4 *s = slot + (DB == 2 ? (j & 1) * 1536 : 0) + lane;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        u32x4 v[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) v[q] = s[(w * 6 + q) * 64];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t voff = tile_voff(tile, w * 64 + lane);
#pragma unroll
        for (int o = 0; o < 3; ++o) {
          gstore<SPOL>(out[o], voff, v[o * 2]);
          gstore<SPOL>(out[o], voff + 32, v[o * 2 + 1]);
        }
      }
      // DB == 2: buffer j&1 is rewritten by tile j+2, whose B barrier comes
      // after tile j+1's B, which this wave joins only after these reads.
    }
  }
}

int main(int argc, char **argv) {
  const uint32_t K = 30, B = 4;
  const uint64_t S = 32ull << 20;
  uint8_t *data, *par;
  CHECK(hipMalloc(&data, S * K * B));
  CHECK(hipMalloc(&par, S * 3 * B));
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
  const double rs_bytes = double(S) * (K + 3) * B, rd_bytes = double(S) * K * B;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const uint32_t total = tpb * B;
  {  // clock settle
    for (int i = 0; i < 600; ++i)
      hipLaunchKernelGGL((base_probe<1>), dim3(total), dim3(256), 0, 0, a);
    CHECK(hipDeviceSynchronize());
    printf("{\"settle\": \"ok\"}\n");
    fflush(stdout);
  }
  auto time = [&](const char *name, auto launch, double nbytes) {
    fprintf(stderr, "start %s\n", name);
    for (int i = 0; i < 5; ++i) launch();
    CHECK(hipDeviceSynchronize());
    const int iters = 30;
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
  time("ro", [&] { hipLaunchKernelGGL((base_probe<0>), dim3(total), dim3(256), 0, 0, a); }, rd_bytes);

  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
#define WW(DB, SP)                                                                            \
  do {                                                                                        \
    const size_t lds = size_t(DB) * 24576;                                                    \
    int per = 0;                                                                              \
    auto kfn = ww_probe<DB, SP>;                                                              \
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, 320, lds));                 \
    for (int f = per; f >= 1 && f >= per - 2; --f) {                                          \
      const uint32_t G = uint32_t(f * ncu);                                                   \
      char name[64];                                                                          \
      snprintf(name, sizeof name, "ww_db%d_s%d_per%d", DB, SP, f);                            \
      time(name, [&] { hipLaunchKernelGGL((ww_probe<DB, SP>), dim3(G), dim3(320), lds, 0, a); }, \
           rs_bytes);                                                                         \
    }                                                                                         \
  } while (0)
  WW(1, 1);
  WW(1, 0);
  WW(2, 1);
  WW(2, 0);
  time("base_again", [&] { hipLaunchKernelGGL((base_probe<1>), dim3(total), dim3(256), 0, 0, a); }, rs_bytes);
  return 0;
}
