// membench2.hip — HBM pattern probes for the RS(30,3) pass, round 2
// (measurement tool, not product code).  Every rs_probe reads K=30 input
// shards and writes 3 output shards per block (4 blocks, 32 MiB shards) with
// the product kernel's lane layout (lane = 32-byte half-chunk: 16 B at +0 and
// 16 B at +32, 8 KiB tile per 256-lane workgroup, 3 inputs in flight), XOR
// in place of the GF arithmetic.  Knobs:
//   GRID    0 = one workgroup per tile (product), 1 = persistent grid-stride,
//           2 = persistent contiguous tile ranges
//   LPOL    load cache policy: 0 none, 1 nt, 2 sc1
//   SPOL    store cache policy: 0 none, 1 nt, 2 sc0 sc1
//   WRITES  0 = reads only (30 streams), 1 = 30 reads + 3 writes
// Also: float4 copy / read kernels with U loads in flight per lane.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/membench2.hip -o tools/membench2
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));           \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Shard addresses travel in the kernarg segment (as in the product kernel):
// the compiler fetches them with s_load (SMEM), never through a VALU write of
// an SGPR.  A v_readfirstlane-produced SGPR used as the saddr of the next
// inline-asm VMEM instruction is a hazard (5 wait states) the compiler does
// not see inside asm: the first version of this probe did that and faulted.
struct Args {
  uint64_t in[120];  // K * B shard addresses
  uint64_t out[12];  // 3 * B
  uint32_t K, B;
  uint32_t tiles_per_block;  // S / 8 KiB
  uint32_t total_tiles;      // tiles_per_block * B
};

template <int LPOL>
__device__ __forceinline__ void gload2(u32x4 &L, u32x4 &H, uint64_t base, uint32_t voff) {
  if constexpr (LPOL == 0)
    asm volatile("global_load_dwordx4 %0, %2, %3\n\tglobal_load_dwordx4 %1, %2, %3 offset:32"
                 : "=&v"(L), "=&v"(H) : "v"(voff), "s"(base) : "memory");
  else if constexpr (LPOL == 1)
    asm volatile("global_load_dwordx4 %0, %2, %3 nt\n\tglobal_load_dwordx4 %1, %2, %3 offset:32 nt"
                 : "=&v"(L), "=&v"(H) : "v"(voff), "s"(base) : "memory");
  else
    asm volatile("global_load_dwordx4 %0, %2, %3 sc1\n\tglobal_load_dwordx4 %1, %2, %3 offset:32 sc1"
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
  else if constexpr (SPOL == 1)
    asm volatile("global_store_dwordx4 %0, %1, %2 nt" ::"v"(voff), "v"(v), "s"(base) : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, %2 sc0 sc1" ::"v"(voff), "v"(v), "s"(base) : "memory");
}

template <int LPOL, int SPOL, int WRITES>
__device__ __forceinline__ void do_tile(const Args &a, uint32_t t, uint32_t wave) {
  const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
  const uint64_t hc = uint64_t(tile) * 256 + threadIdx.x;
  const uint32_t voff = uint32_t((hc >> 1) * 64 + (hc & 1) * 16);
  const uint64_t *in = a.in + b * a.K;
  const uint32_t K = a.K;
  const uint32_t rot = (tile * 4 + wave) % K;
  auto idx = [&](uint32_t x) -> uint32_t {
    if (x >= K) x = K - 1;
    const uint32_t y = rot + x;
    return y >= K ? y - K : y;
  };
  u32x4 accL = {0, 0, 0, 0}, accH = {0, 0, 0, 0};
  u32x4 LA, HA, LB, HB, LC, HC, LD, HD;
  gload2<LPOL>(LA, HA, in[idx(0)], voff);
  gload2<LPOL>(LB, HB, in[idx(1)], voff);
  gload2<LPOL>(LC, HC, in[idx(2)], voff);
  for (uint32_t i = 0;; i += 4) {
    gload2<LPOL>(LD, HD, in[idx(i + 3)], voff);
    vm_wait<6>(LA, HA);
    accL ^= LA; accH ^= HA;
    gload2<LPOL>(LA, HA, in[idx(i + 4)], voff);
    vm_wait<6>(LB, HB);
    accL ^= LB; accH ^= HB;
    if (i + 2 >= K) break;
    gload2<LPOL>(LB, HB, in[idx(i + 5)], voff);
    vm_wait<6>(LC, HC);
    accL ^= LC; accH ^= HC;
    gload2<LPOL>(LC, HC, in[idx(i + 6)], voff);
    vm_wait<6>(LD, HD);
    accL ^= LD; accH ^= HD;
    if (i + 4 >= K) break;
  }
  vm_wait<0>(LA, HA);
  if constexpr (WRITES) {
    const uint64_t *out = a.out + b * 3;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      gstore<SPOL>(out[o], voff, accL + u32x4{uint32_t(o), 0, 0, 0});
      gstore<SPOL>(out[o], voff + 32, accH + u32x4{uint32_t(o), 0, 0, 0});
    }
  } else {
    if (accL.x == 0x12345678u && accH.y == 0x9abcdef0u) gstore<0>(a.out[0], voff, accL);
  }
}

template <int GRID, int LPOL, int SPOL, int WRITES>
__global__ __launch_bounds__(256) void rs_probe(const Args a) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (GRID == 0) {
    do_tile<LPOL, SPOL, WRITES>(a, blockIdx.x, wave);
  } else if constexpr (GRID == 1) {
    for (uint32_t t = blockIdx.x; t < a.total_tiles; t += gridDim.x)
      do_tile<LPOL, SPOL, WRITES>(a, t, wave);
  } else {
    const uint32_t per = (a.total_tiles + gridDim.x - 1) / gridDim.x;
    const uint32_t t0 = blockIdx.x * per, t1 = min(t0 + per, a.total_tiles);
    for (uint32_t t = t0; t < t1; ++t) do_tile<LPOL, SPOL, WRITES>(a, t, wave);
  }
}

// Write-only: the RS store pattern alone (3 output shards, 8 KiB tile per
// workgroup, two 16-B stores per lane per output).
template <int SPOL>
__global__ __launch_bounds__(256) void ws_probe(const Args a) {
  const uint32_t t = blockIdx.x;
  const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
  const uint64_t hc = uint64_t(tile) * 256 + threadIdx.x;
  const uint32_t voff = uint32_t((hc >> 1) * 64 + (hc & 1) * 16);
  const u32x4 v = {t, threadIdx.x, 1, 2};
  const uint64_t *out = a.out + b * 3;
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    gstore<SPOL>(out[o], voff, v);
    gstore<SPOL>(out[o], voff + 32, v);
  }
}

// Coarse bursts: a workgroup reads T consecutive tiles (keeping T tiles of
// outputs in registers), then writes all T tiles' outputs together.
template <int T, int SPOL>
__global__ __launch_bounds__(256) void burst_probe(const Args a) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t t0 = blockIdx.x * T;
  const uint32_t b = t0 / a.tiles_per_block;
  const uint64_t *in = a.in + b * a.K;
  const uint32_t K = a.K;
  u32x4 accL[T], accH[T];
  uint32_t voffs[T];
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const uint32_t tile = t0 + j - b * a.tiles_per_block;
    const uint64_t hc = uint64_t(tile) * 256 + threadIdx.x;
    const uint32_t voff = uint32_t((hc >> 1) * 64 + (hc & 1) * 16);
    voffs[j] = voff;
    const uint32_t rot = (tile * 4 + wave) % K;
    auto idx = [&](uint32_t x) -> uint32_t {
      if (x >= K) x = K - 1;
      const uint32_t y = rot + x;
      return y >= K ? y - K : y;
    };
    u32x4 aL = {0, 0, 0, 0}, aH = {0, 0, 0, 0};
    u32x4 LA, HA, LB, HB, LC, HC, LD, HD;
    gload2<0>(LA, HA, in[idx(0)], voff);
    gload2<0>(LB, HB, in[idx(1)], voff);
    gload2<0>(LC, HC, in[idx(2)], voff);
    for (uint32_t i = 0;; i += 4) {
      gload2<0>(LD, HD, in[idx(i + 3)], voff);
      vm_wait<6>(LA, HA);
      aL ^= LA; aH ^= HA;
      gload2<0>(LA, HA, in[idx(i + 4)], voff);
      vm_wait<6>(LB, HB);
      aL ^= LB; aH ^= HB;
      if (i + 2 >= K) break;
      gload2<0>(LB, HB, in[idx(i + 5)], voff);
      vm_wait<6>(LC, HC);
      aL ^= LC; aH ^= HC;
      gload2<0>(LC, HC, in[idx(i + 6)], voff);
      vm_wait<6>(LD, HD);
      aL ^= LD; aH ^= HD;
      if (i + 4 >= K) break;
    }
    vm_wait<0>(LA, HA);
    accL[j] = aL;
    accH[j] = aH;
  }
  const uint64_t *out = a.out + b * 3;
#pragma unroll
  for (int j = 0; j < T; ++j)
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      gstore<SPOL>(out[o], voffs[j], accL[j] + u32x4{uint32_t(o), 0, 0, 0});
      gstore<SPOL>(out[o], voffs[j] + 32, accH[j] + u32x4{uint32_t(o), 0, 0, 0});
    }
}

// float4 copy with U independent 16-B loads in flight per lane per iteration.
template <int U, int LPOL, int SPOL>
__global__ __launch_bounds__(256) void copy_u(const u32x4 *__restrict__ s, u32x4 *__restrict__ d,
                                              size_t n) {
  const size_t stride = size_t(gridDim.x) * 256;
  for (size_t base = size_t(blockIdx.x) * 256 * U; base < n; base += stride * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * 256 + threadIdx.x;
      if (LPOL == 1)
        v[u] = __builtin_nontemporal_load(s + (i < n ? i : 0));
      else
        v[u] = s[i < n ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * 256 + threadIdx.x;
      if (i < n) {
        if (SPOL == 1)
          __builtin_nontemporal_store(v[u], d + i);
        else
          d[i] = v[u];
      }
    }
  }
}

template <int U, int LPOL>
__global__ __launch_bounds__(256) void read_u(const u32x4 *__restrict__ s, u32x4 *__restrict__ d,
                                              size_t n) {
  const size_t stride = size_t(gridDim.x) * 256;
  u32x4 acc = {0, 0, 0, 0};
  for (size_t base = size_t(blockIdx.x) * 256 * U; base < n; base += stride * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * 256 + threadIdx.x;
      acc ^= (LPOL == 1) ? __builtin_nontemporal_load(s + (i < n ? i : 0)) : s[i < n ? i : 0];
    }
  }
  if (acc.x == 0x12345678u) d[0] = acc;
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
  // clock settle: ~1 s of streaming before any measurement
  {
    const size_t n = S * K * B / 16;
    for (int i = 0; i < 200; ++i)
      hipLaunchKernelGGL((read_u<4, 0>), dim3(2048), dim3(256), 0, 0, (const u32x4 *)data,
                         (u32x4 *)par, n);
    CHECK(hipDeviceSynchronize());
    printf("{\"settle\": \"ok\"}\n");
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
  const uint32_t total = tpb * B;
#define RS(GRID, LP, SP, WR, G)                                                                     \
  time("rs_grid" #GRID "_g" #G "_l" #LP "_s" #SP "_w" #WR,                                          \
       [&] {                                                                                       \
         hipLaunchKernelGGL((rs_probe<GRID, LP, SP, WR>), dim3(GRID == 0 ? total : (G)), dim3(256), \
                            0, 0, a);                                                              \
       },                                                                                          \
       WR ? rs_bytes : rd_bytes)
  RS(0, 0, 1, 1, 0);  // the product's pattern
  RS(0, 1, 1, 1, 0);
  RS(0, 2, 1, 1, 0);
  RS(0, 0, 0, 1, 0);
  RS(0, 0, 2, 1, 0);
  RS(0, 1, 0, 1, 0);
  RS(0, 0, 1, 0, 0);  // reads only
  RS(0, 1, 1, 0, 0);
  RS(1, 0, 1, 1, 2048);
  RS(1, 1, 1, 1, 2048);
  RS(1, 0, 1, 1, 4096);
  RS(1, 1, 1, 1, 4096);
  RS(2, 0, 1, 1, 2048);
  RS(2, 1, 1, 1, 2048);
  RS(2, 1, 0, 1, 2048);
  RS(1, 0, 1, 1, 1024);
  RS(1, 1, 1, 0, 2048);
  RS(0, 0, 1, 1, 0);  // repeat baseline (drift check)

  const double ws_bytes = double(S) * 3 * B;
  time("write_only_s1", [&] { hipLaunchKernelGGL((ws_probe<1>), dim3(total), dim3(256), 0, 0, a); }, ws_bytes);
  time("write_only_s0", [&] { hipLaunchKernelGGL((ws_probe<0>), dim3(total), dim3(256), 0, 0, a); }, ws_bytes);
  time("burst_t2_s1", [&] { hipLaunchKernelGGL((burst_probe<2, 1>), dim3(total / 2), dim3(256), 0, 0, a); }, rs_bytes);
  time("burst_t4_s1", [&] { hipLaunchKernelGGL((burst_probe<4, 1>), dim3(total / 4), dim3(256), 0, 0, a); }, rs_bytes);
  time("burst_t4_s0", [&] { hipLaunchKernelGGL((burst_probe<4, 0>), dim3(total / 4), dim3(256), 0, 0, a); }, rs_bytes);
  RS(0, 0, 1, 1, 0);  // baseline again

  const size_t n = S * K * B / 2 / 16;  // copy: first half of `data` -> second half
#define CP(U, LP, SP, G)                                                                     \
  time("copy_u" #U "_l" #LP "_s" #SP "_g" #G,                                                \
       [&] {                                                                                 \
         hipLaunchKernelGGL((copy_u<U, LP, SP>), dim3(G), dim3(256), 0, 0, (const u32x4 *)data, \
                            (u32x4 *)(data + n * 16), n);                                     \
       },                                                                                    \
       2.0 * n * 16)
  CP(1, 0, 0, 2048);
  CP(4, 0, 0, 2048);
  CP(4, 1, 1, 2048);
  CP(4, 0, 1, 2048);
  CP(8, 1, 1, 2048);
  CP(4, 1, 1, 4096);
  const size_t nr = S * K * B / 16;
#define RD(U, LP, G)                                                                          \
  time("read_u" #U "_l" #LP "_g" #G,                                                          \
       [&] { hipLaunchKernelGGL((read_u<U, LP>), dim3(G), dim3(256), 0, 0, (const u32x4 *)data, \
                                (u32x4 *)par, nr); },                                         \
       double(nr) * 16)
  RD(4, 0, 2048);
  RD(4, 1, 2048);
  RD(8, 1, 2048);
  RD(8, 1, 4096);
  return 0;
}
