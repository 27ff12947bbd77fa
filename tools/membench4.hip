// membench4.hip — locality probes for the RS(30,3) pass (measurement tool,
// not product code).
//
// Question: the product pattern (30 read streams + 3 write streams, one
// workgroup per 8 KiB tile, waves rotated over inputs) reads 6.35 TB/s alone
// but 5.0-5.2 TB/s with its 9% of writes, while a float4 copy (50% writes)
// reaches 6.3.  A persistent grid of ONE workgroup per CU ran faster than the
// full-occupancy grid (membench3): is it DRAM locality (how many distinct
// rows the chip touches at once) rather than latency?
//
// Knobs: ROT (which input each wave reads first), occupancy cap (dynamic LDS
// per workgroup), persistent grid-stride grid size, writes on/off.
//   ROT 0: none; 1: (tile*4+wave)%K (product); 2: tile%K (whole WG together);
//       3: ((tile>>4)*4+wave)%K; 4: (tile>>4)%K; 5: (wave*8)%K
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/membench4.hip -o tools/membench4
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
template <int ROT>
__device__ __forceinline__ void read_tile(const Args &a, uint32_t t, uint32_t wave, uint32_t lane256,
                                          u32x4 &accL, u32x4 &accH) {
  const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
  const uint32_t voff = tile_voff(tile, lane256);
  const uint64_t *in = a.in + b * a.K;
  const uint32_t K = a.K;
  uint32_t rot;
  if (ROT == 0) rot = 0;
  else if (ROT == 1) rot = (tile * 4 + wave) % K;
  else if (ROT == 2) rot = tile % K;
  else if (ROT == 3) rot = ((tile >> 4) * 4 + wave) % K;
  else if (ROT == 4) rot = (tile >> 4) % K;
  else rot = (wave * 8) % K;
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


template <int ROT, int WRITES, int SPOL>
__global__ __launch_bounds__(256) void probe(const Args a) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint32_t t = blockIdx.x; t < a.total_tiles; t += gridDim.x) {
    u32x4 accL, accH;
    read_tile<ROT>(a, t, wave, threadIdx.x, accL, accH);
    const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
    const uint32_t voff = tile_voff(tile, threadIdx.x);
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
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  {  // clock settle
    for (int i = 0; i < 600; ++i)
      hipLaunchKernelGGL((probe<1, 1, 1>), dim3(total), dim3(256), 0, 0, a);
    CHECK(hipDeviceSynchronize());
    printf("{\"settle\": \"ok\"}\n");
    fflush(stdout);
  }
  auto time = [&](const char *name, auto launch, double nbytes) {
    fprintf(stderr, "start %s\n", name);
    for (int i = 0; i < 5; ++i) launch();
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
  // occ: dynamic LDS caps workgroups per CU (160 KiB / lds); G: 0 = one WG per tile
  auto run = [&](auto kfn, const char *tag, int rot, int wr, int sp, size_t lds, uint32_t per_cu) {
    const uint32_t G = per_cu ? per_cu * uint32_t(ncu) : total;
    char name[96];
    snprintf(name, sizeof name, "%s_rot%d_w%d_s%d_lds%zuk_g%u", tag, rot, wr, sp, lds >> 10, per_cu);
    time(name, [&] { hipLaunchKernelGGL(kfn, dim3(G), dim3(256), lds, 0, a); }, wr ? rs_bytes : rd_bytes);
  };
#define SWEEP(ROT)                                                                 \
  do {                                                                             \
    auto kw = probe<ROT, 1, 1>;                                                    \
    auto kp = probe<ROT, 1, 0>;                                                    \
    auto kr = probe<ROT, 0, 1>;                                                    \
    run(kw, "t", ROT, 1, 1, 0, 0);                                                 \
    run(kp, "t", ROT, 1, 0, 0, 0);                                                 \
    run(kr, "t", ROT, 0, 1, 0, 0);                                                 \
    run(kw, "t", ROT, 1, 1, 56 << 10, 0);                                          \
    run(kw, "t", ROT, 1, 1, 96 << 10, 0);                                          \
    run(kw, "p", ROT, 1, 1, 96 << 10, 1);                                          \
    run(kp, "p", ROT, 1, 0, 96 << 10, 1);                                          \
    run(kw, "p", ROT, 1, 1, 56 << 10, 2);                                          \
    run(kw, "p", ROT, 1, 1, 0, 4);                                                 \
  } while (0)
  SWEEP(1);
  SWEEP(0);
  SWEEP(2);
  SWEEP(3);
  SWEEP(4);
  SWEEP(5);
  run(probe<1, 1, 1>, "again", 1, 1, 1, 0, 0);
  return 0;
}
