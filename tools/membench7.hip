// membench7.hip — lockstep probes for the RS(30,3) pass (measurement tool,
// not product code).
//
// membench5: the marginal cost of the parity writes grows with the number of
// read streams (k3: 5.6 TB/s marginal, k10: 4, k30: 1.6).  Hypothesis: what
// matters is how many distinct DRAM windows the whole chip touches at once.
// These probes make every CU read the SAME input shard at the same time: a
// persistent grid (1 workgroup per CU), each workgroup owning NW/4
// consecutive 8 KiB tiles (a "super-tile"), inputs in order 0..K-1 with no
// rotation, and (SYNC) a grid-wide barrier every SYNC super-tiles.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/membench7.hip -o tools/membench7
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

template <int NW, int SYNC, int ROT>
__global__ __launch_bounds__(NW * 64) void lockstep(const Args a, uint32_t *cnt) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t grp = wave >> 2, w4 = wave & 3, l256 = threadIdx.x & 255;
  const uint32_t G = gridDim.x, total_st = a.total_tiles / (NW / 4);
  uint32_t round = 0;
  for (uint32_t st = blockIdx.x; st < total_st; st += G, ++round) {
    if (SYNC && round > 0 && round % SYNC == 0) {
      asm volatile("s_barrier" ::: "memory");
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        spin_until(cnt, G * (round / SYNC));
      }
      asm volatile("s_barrier" ::: "memory");
    }
    const uint32_t t = st * (NW / 4) + grp;
    const uint32_t b = t / a.tiles_per_block, tile = t - b * a.tiles_per_block;
    const uint32_t voff = tile_voff(tile, l256);
    const uint64_t *in = a.in + b * a.K;
    const uint32_t K = a.K;
    const uint32_t rot = ROT ? (tile * 4 + w4) % K : 0;
    auto idx = [&](uint32_t x) -> uint32_t {
      if (x >= K) x = K - 1;
      const uint32_t y = rot + x;
      return y >= K ? y - K : y;
    };
    u32x4 accL = {0, 0, 0, 0}, accH = {0, 0, 0, 0};
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
    const uint64_t *out = a.out + b * 3;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      gstore<1>(out[o], voff, accL + u32x4{uint32_t(o), 0, 0, 0});
      gstore<1>(out[o], voff + 32, accH + u32x4{uint32_t(o), 0, 0, 0});
    }
  }
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
  auto run = [&](auto kfn, int nw, int sync, int rot, int per_cu) {
    int per = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, nw * 64, 0));
    if (per < per_cu) { printf("{\"skip\": %d}\n", nw); return; }
    const uint32_t G = uint32_t(per_cu * ncu);
    char name[96];
    snprintf(name, sizeof name, "ls_nw%d_sync%d_rot%d_per%d", nw, sync, rot, per_cu);
    time(name, [&] {
      (void)hipMemsetAsync(cnt, 0, 4096, 0);
      hipLaunchKernelGGL(kfn, dim3(G), dim3(nw * 64), 0, 0, a, cnt);
    }, rs_bytes);
  };
  run(lockstep<16, 0, 0>, 16, 0, 0, 1);
  run(lockstep<16, 1, 0>, 16, 1, 0, 1);
  run(lockstep<16, 2, 0>, 16, 2, 0, 1);
  run(lockstep<16, 4, 0>, 16, 4, 0, 1);
  run(lockstep<16, 1, 1>, 16, 1, 1, 1);
  run(lockstep<16, 0, 1>, 16, 0, 1, 1);
  run(lockstep<8, 0, 0>, 8, 0, 0, 2);
  run(lockstep<8, 1, 0>, 8, 1, 0, 2);
  run(lockstep<16, 0, 0>, 16, 0, 0, 2);
  run(lockstep<16, 1, 0>, 16, 1, 0, 2);
  run(lockstep<4, 0, 0>, 4, 0, 0, 4);
  run(lockstep<4, 1, 0>, 4, 1, 0, 4);
  time("base_again", [&] { hipLaunchKernelGGL((base_probe<1>), dim3(total), dim3(256), 0, 0, a); }, rs_bytes);
  return 0;
}
