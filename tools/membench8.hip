// membench8.hip — round-2 HBM probes for the RS(k,3) pass (measurement tool,
// not product code; traffic only, the XORed values are meaningless).
//
// Question: the RS pattern (30 read streams + 3 write streams per block) runs
// at ~5.0-5.2 TB/s in traffic-only form while one read stream runs 7.1 TB/s
// and a one-stream copy ~7.0 TB/s (profiles/r01v_membench/mb5.jsonl).  This
// probe varies what round 1 did not: the contiguous run one wave reads from a
// stream per step (NL x 1 KiB), the ring depth (streams in flight), and
// register vs LDS-DMA staging, at a constant 120 x 32 MiB of reads.
//
// Generic probe P<K, O, NL, HC, NTL, NTS, D, XG>: a workgroup (4 waves) owns
// 4*NL KiB of columns of every shard of one block of K input shards; it XORs
// the K inputs (D+1 inputs in flight per wave) and stores the result into the
// block's O outputs.  HC = product lane layout (16 B at +0 / +32 of a 64-B
// chunk per load pair) instead of contiguous 1 KiB per load instruction.
// Read order: groups of 16 tiles share a starting input (product v41); XG=1
// places a group's 16 workgroups on one XCD (product v58).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/membench8.hip -o tools/membench8
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <chrono>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));           \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define AS_CONST __attribute__((address_space(4)))

constexpr uint64_t kS = 32ull << 20;  // shard bytes
constexpr uint32_t kShards = 120;     // input shards of every probe

struct Args {
  const uint64_t *in;   // B*K shard addresses (device array)
  const uint64_t *out;  // B*O shard addresses
  uint32_t tiles_per_block;
  uint32_t total_tiles;
};

template <int NTL>
__device__ __forceinline__ void gload(u32x4 &v, uint64_t base, uint32_t voff) {
  if constexpr (NTL)
    asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=&v"(v) : "v"(voff), "s"(base) : "memory");
  else
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=&v"(v) : "v"(voff), "s"(base) : "memory");
}

template <int NTS>
__device__ __forceinline__ void gstore(uint64_t base, uint32_t voff, const u32x4 &v) {
  if constexpr (NTS)
    asm volatile("global_store_dwordx4 %0, %1, %2 nt" ::"v"(voff), "v"(v), "s"(base) : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, %2" ::"v"(voff), "v"(v), "s"(base) : "memory");
}

__device__ __forceinline__ void axor(u32x4 &acc, const u32x4 &v) {
  // asm so the XORs stay in program order (the compiler would otherwise sink
  // them to the end and keep every buffer live)
  asm volatile("v_xor_b32 %0, %0, %4\n\tv_xor_b32 %1, %1, %5\n\tv_xor_b32 %2, %2, %6\n\tv_xor_b32 %3, %3, %7"
               : "+v"(acc.x), "+v"(acc.y), "+v"(acc.z), "+v"(acc.w)
               : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
}

template <int N, int NL>
__device__ __forceinline__ void wait_buf(u32x4 (&b)[NL]) {
  // every register of the buffer is an in/out operand: nothing reads it above the wait
  if constexpr (NL == 2)
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(b[0]), "+v"(b[1]) : "n"(N) : "memory");
  else if constexpr (NL == 4)
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) : "n"(N)
                 : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]),
                   "+v"(b[6]), "+v"(b[7])
                 : "n"(N)
                 : "memory");
}

__device__ __forceinline__ uint32_t xcd_remap16(uint32_t b, uint32_t n) {
  constexpr uint32_t XG = 16, run = 8 * XG;
  const uint32_t full = n / run * run;
  if (b >= full) return b;
  const uint32_t base = b / run * run, r = b - base, x = r & 7u, q = r >> 3;
  return base + XG * (8u * (q / XG) + x) + q % XG;
}

// HC = 2: contiguous 1 KiB per instruction but the product v70/71 lane order
// (lanes 0-31 the low 32-B halves of 16 chunks, lanes 32-63 the high halves):
// same bytes per instruction, consecutive lanes 32 B apart.
template <int NL, int HC>
__device__ __forceinline__ uint32_t lane_off(uint32_t col0, uint32_t lane, int j) {
  if constexpr (HC == 2) {
    return col0 + uint32_t(j) * 1024 + ((lane & 31) >> 1) * 64 + (lane >> 5) * 32 + (lane & 1) * 16;
  } else if constexpr (HC) {
    // pairs of loads: (lo 16 B at +0, hi 16 B at +32) of half-chunk (j/2)*64 + lane
    const uint32_t hc = uint32_t(j / 2) * 64 + lane;
    return col0 + (hc >> 1) * 64 + (hc & 1) * 16 + uint32_t(j & 1) * 32;
  } else {
    return col0 + uint32_t(j) * 1024 + lane * 16;
  }
}

// PRO = 1: the product kernel's prologue first (enter_pass: 30 inputs x 512 B
// of nibble tables from a global buffer into LDS, then a barrier).

template <int K, int O, int NL, int HC, int NTL, int NTS, int D, int XG, int PRO = 0, int WAVES = 4>
__global__ __launch_bounds__(64 * WAVES) void probe(Args a) {
  if constexpr (PRO) {
    extern __shared__ __attribute__((aligned(16))) u32x4 tab_lds[];
    const u32x4 *tab = (const u32x4 *)a.out;  // any resident bytes: 960 x 16 B
    u32x4 v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t e = threadIdx.x + 256u * r;
      v[r] = e < 960 ? tab[e] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t e = threadIdx.x + 256u * r;
      if (e < 960) tab_lds[e] = v[r];
    }
    __syncthreads();
  }
  const uint32_t wg = XG ? xcd_remap16(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t blk = wg / a.tiles_per_block, tile = wg % a.tiles_per_block;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t col0 = (tile * WAVES + wave) * NL * 1024;
  const AS_CONST uint64_t *in = (const AS_CONST uint64_t *)(uintptr_t)(a.in + size_t(blk) * K);
  const uint32_t rot = K > 1 ? ((tile >> 4) * 4) % K : 0;
  u32x4 buf[K][NL];
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < K + D + 1; ++i) {
    if (i < K) {  // issue input i
      const uint32_t s = (rot + i) % K;
      const uint64_t base = in[s];
#pragma unroll
      for (int j = 0; j < NL; ++j) gload<NTL>(buf[i][j], base, lane_off<NL, HC>(col0, lane, j));
    }
    const int c = i - D;  // consume input c: loads issued after it = min(D, K-1-c) inputs
    if (c >= 0 && c < K) {
      const int after = (K - 1 - c) < D ? (K - 1 - c) : D;
      switch (after * NL) {  // compile-time after full unroll
        case 0: wait_buf<0, NL>(buf[c]); break;
        case 2: wait_buf<2, NL>(buf[c]); break;
        case 4: wait_buf<4, NL>(buf[c]); break;
        case 6: wait_buf<6, NL>(buf[c]); break;
        case 8: wait_buf<8, NL>(buf[c]); break;
        case 12: wait_buf<12, NL>(buf[c]); break;
        case 16: wait_buf<16, NL>(buf[c]); break;
        case 24: wait_buf<24, NL>(buf[c]); break;
        case 32: wait_buf<32, NL>(buf[c]); break;
        case 48: wait_buf<48, NL>(buf[c]); break;
        default: wait_buf<0, NL>(buf[c]); break;
      }
#pragma unroll
      for (int j = 0; j < NL; ++j) axor(acc, buf[c][j]);
    }
  }
  if constexpr (O > 0) {
    const AS_CONST uint64_t *out =
        (const AS_CONST uint64_t *)(uintptr_t)(a.out + size_t(blk) * O);
#pragma unroll
    for (int o = 0; o < O; ++o) {
      const uint64_t base = out[o];
#pragma unroll
      for (int j = 0; j < NL; ++j)
        gstore<NTS>(base, lane_off<NL, HC>(col0, lane, j), acc + u32x4{uint32_t(o + j), 0, 0, 0});
    }
  } else {
    if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) {  // never: keeps the loads alive
      *(u32x4 *)(uintptr_t)(a.out[0] + lane * 16) = acc;
    }
  }
}

// LDS-DMA staging variant: each wave streams its NL KiB run of input i into an
// LDS ring slot with global_load_lds_dwordx4 (M0 = slot base), D+1 slots per
// wave, then reads it back with ds_read_b128.  Traffic-only like `probe`.
template <int K, int O, int NL, int NTL, int NTS, int D, int WAVES = 4>
__global__ __launch_bounds__(64 * WAVES) void probe_lds(Args a) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const uint32_t wg = xcd_remap16(blockIdx.x, gridDim.x);
  const uint32_t blk = wg / a.tiles_per_block, tile = wg % a.tiles_per_block;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t col0 = (tile * WAVES + wave) * NL * 1024;
  const AS_CONST uint64_t *in = (const AS_CONST uint64_t *)(uintptr_t)(a.in + size_t(blk) * K);
  const uint32_t rot = K > 1 ? ((tile >> 4) * 4) % K : 0;
  // per-wave ring of D+1 slots of NL KiB
  const uint32_t wave_lds = wave * (D + 1) * NL * 1024;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < K + D + 1; ++i) {
    if (i < K) {
      const uint32_t s = (rot + i) % K;
      const uint64_t base = in[s];
      const uint32_t slot = wave_lds + uint32_t(i % (D + 1)) * NL * 1024;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const uint32_t m0 = slot + uint32_t(j) * 1024;
        const uint32_t voff = col0 + uint32_t(j) * 1024 + lane * 16;
        uint32_t keep;
        if constexpr (NTL)
          asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                       "global_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                       : "=&s"(keep) : "v"(voff), "s"(base), "s"(m0) : "memory");
        else
          asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                       "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                       : "=&s"(keep) : "v"(voff), "s"(base), "s"(m0) : "memory");
      }
    }
    const int c = i - D;
    if (c >= 0 && c < K) {
      const int after = (K - 1 - c) < D ? (K - 1 - c) : D;
      switch (after * NL) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
        case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
        case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
        case 48: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }
      const uint32_t slot = wave_lds + uint32_t(c % (D + 1)) * NL * 1024;
#pragma unroll
      for (int j = 0; j < NL; ++j) axor(acc, lds[(slot + uint32_t(j) * 1024) / 16 + lane]);
      // the slot is refilled D+1 inputs later by this wave only: the ds_reads
      // above must finish first
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  if constexpr (O > 0) {
    const AS_CONST uint64_t *out =
        (const AS_CONST uint64_t *)(uintptr_t)(a.out + size_t(blk) * O);
#pragma unroll
    for (int o = 0; o < O; ++o) {
      const uint64_t base = out[o];
#pragma unroll
      for (int j = 0; j < NL; ++j)
        gstore<NTS>(base, col0 + uint32_t(j) * 1024 + lane * 16, acc + u32x4{uint32_t(o + j), 0, 0, 0});
    }
  } else {
    if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u)
      *(u32x4 *)(uintptr_t)(a.out[0] + lane * 16) = acc;
  }
}

// Round 6 (tiled layout question): the same traffic with each block's shards
// stored tile-major -- for tile t of block b, the K input pieces of WG bytes
// (and, INTER=1, the O output pieces) sit next to each other -- so the chip
// reads one near-sequential stream instead of K streams 32 MiB apart.  No read
// rotation (the pieces are read in address order).
struct TArgs {
  uint64_t data, out;
  uint32_t tiles_per_block, total_tiles;
};

template <int K, int O, int NL, int NTL, int NTS, int D, int INTER, int XG, int WAVES = 4>
__global__ __launch_bounds__(64 * WAVES) void probe_tiled(TArgs a) {
  const uint32_t wg = XG ? xcd_remap16(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr uint32_t WGB = WAVES * NL * 1024;
  constexpr uint32_t P = INTER ? K + O : K;  // pieces per tile in the data region
  const uint64_t region = a.data + uint64_t(wg) * P * WGB;
  const uint32_t off0 = wave * NL * 1024 + lane * 16;
  u32x4 buf[K][NL];
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < K + D + 1; ++i) {
    if (i < K) {
      const uint64_t base = region + uint64_t(i) * WGB;
#pragma unroll
      for (int j = 0; j < NL; ++j) gload<NTL>(buf[i][j], base, off0 + uint32_t(j) * 1024);
    }
    const int c = i - D;
    if (c >= 0 && c < K) {
      const int after = (K - 1 - c) < D ? (K - 1 - c) : D;
      switch (after * NL) {
        case 0: wait_buf<0, NL>(buf[c]); break;
        case 2: wait_buf<2, NL>(buf[c]); break;
        case 4: wait_buf<4, NL>(buf[c]); break;
        case 6: wait_buf<6, NL>(buf[c]); break;
        case 8: wait_buf<8, NL>(buf[c]); break;
        case 12: wait_buf<12, NL>(buf[c]); break;
        case 16: wait_buf<16, NL>(buf[c]); break;
        default: wait_buf<0, NL>(buf[c]); break;
      }
#pragma unroll
      for (int j = 0; j < NL; ++j) axor(acc, buf[c][j]);
    }
  }
  if constexpr (O > 0) {
#pragma unroll
    for (int o = 0; o < O; ++o) {
      const uint64_t base =
          INTER ? region + uint64_t(K + o) * WGB : a.out + (uint64_t(wg) * O + o) * WGB;
#pragma unroll
      for (int j = 0; j < NL; ++j)
        gstore<NTS>(base, off0 + uint32_t(j) * 1024, acc + u32x4{uint32_t(o + j), 0, 0, 0});
    }
  } else {
    if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u)
      *(u32x4 *)(uintptr_t)(a.out + lane * 16) = acc;
  }
}

struct Bufs {
  uint8_t *data = nullptr, *outp = nullptr;
  uint64_t pitch = 0;
  uint64_t *d_in = nullptr, *d_out = nullptr;
};

static Bufs g;

template <int K, int O>
Args make_args(uint32_t wg_bytes) {
  constexpr uint32_t B = kShards / K;
  std::vector<uint64_t> hin(B * K), hout(B * (O ? O : 1));
  for (uint32_t i = 0; i < B * K; ++i) hin[i] = uint64_t(g.data + g.pitch * i);
  for (uint32_t i = 0; i < B * (O ? O : 1); ++i) hout[i] = uint64_t(g.outp + g.pitch * i);
  CHECK(hipMemcpy(g.d_in, hin.data(), hin.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(g.d_out, hout.data(), hout.size() * 8, hipMemcpyHostToDevice));
  Args a;
  a.in = g.d_in;
  a.out = g.d_out;
  a.tiles_per_block = uint32_t(kS / wg_bytes);
  a.total_tiles = a.tiles_per_block * B;
  return a;
}

static hipEvent_t e0, e1;

template <typename F>
void timeit(const char *name, F launch, double bytes) {
  // settle: 200 ms of launches, then 3 x 10 timed
  auto t0 = std::chrono::steady_clock::now();
  int n = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.2) {
    launch();
    if (++n % 8 == 0) CHECK(hipDeviceSynchronize());
  }
  CHECK(hipDeviceSynchronize());
  float best = 1e9, sum = 0;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    best = ms < best ? ms : best;
    sum += ms;
  }
  printf("{\"probe\": \"%s\", \"ms\": %.4f, \"mean_ms\": %.4f, \"GBps\": %.1f}\n", name, best,
         sum / 3, bytes / best / 1e6);
  fflush(stdout);
}

// occ > 0: reserve 160 KiB / (occ) of LDS per 4-wave workgroup so at most
// `occ` waves per SIMD run (the product kernel runs 5 at 96 VGPRs)
template <int K, int O, int NL, int HC, int NTL, int NTS, int D, int XG, int PRO = 0, int WAVES = 4>
void run(const char *tag, int occ = 0) {
  constexpr uint32_t B = kShards / K;
  const uint32_t wg_bytes = WAVES * NL * 1024;
  Args a = make_args<K, O>(wg_bytes);
  const double bytes = double(kS) * B * (K + O);
  size_t lds = occ > 0 ? (size_t(160) << 10) / occ / 1024 * 1024 : 0;
  if (PRO && lds < 960 * 16) lds = 960 * 16;
  char name[160];
  snprintf(name, sizeof name, "%s_k%d_o%d_nl%d_%s_ntl%d_nts%d_d%d_xg%d_occ%d_pro%d_w%d", tag, K, O, NL,
           HC == 2 ? "ctperm" : HC ? "hc" : "ct", NTL, NTS, D, XG, occ, PRO, WAVES);
  timeit(name, [&] { hipLaunchKernelGGL((probe<K, O, NL, HC, NTL, NTS, D, XG, PRO, WAVES>), dim3(a.total_tiles),
                                         dim3(64 * WAVES), lds, 0, a); }, bytes);
}

// extra_lds: bytes reserved on top of the ring (the computing kernel's nibble
// tables, 30 x 512 B), so the probe runs at the kernel's workgroups per CU
template <int K, int O, int NL, int NTL, int NTS, int D, int WAVES = 4>
void run_lds(const char *tag, size_t extra_lds = 0) {
  constexpr uint32_t B = kShards / K;
  const uint32_t wg_bytes = WAVES * NL * 1024;
  Args a = make_args<K, O>(wg_bytes);
  const double bytes = double(kS) * B * (K + O);
  const size_t lds = size_t(WAVES) * (D + 1) * NL * 1024 + extra_lds;
  char name[160];
  snprintf(name, sizeof name, "%s_lds_k%d_o%d_nl%d_ntl%d_nts%d_d%d_w%d_x%zu", tag, K, O, NL, NTL,
           NTS, D, WAVES, extra_lds);
  timeit(name, [&] { hipLaunchKernelGGL((probe_lds<K, O, NL, NTL, NTS, D, WAVES>), dim3(a.total_tiles),
                                         dim3(64 * WAVES), lds, 0, a); }, bytes);
}

// tiled probe over a data region of B x tiles x (K [+O]) pieces
template <int K, int O, int NL, int NTL, int NTS, int D, int INTER, int XG, int WAVES = 4>
void run_tiled(const char *tag, uint8_t *data, uint8_t *out, int occ) {
  constexpr uint32_t B = kShards / K;
  const uint32_t wg_bytes = WAVES * NL * 1024;
  TArgs a;
  a.data = uint64_t(data);
  a.out = uint64_t(out);
  a.tiles_per_block = uint32_t(kS / wg_bytes);
  a.total_tiles = a.tiles_per_block * B;
  const double bytes = double(kS) * B * (K + O);
  const size_t lds = occ > 0 ? (size_t(160) << 10) / occ / 1024 * 1024 : 0;
  char name[160];
  snprintf(name, sizeof name, "%s_tiled_k%d_o%d_nl%d_ntl%d_nts%d_d%d_inter%d_xg%d_occ%d_w%d", tag, K, O,
           NL, NTL, NTS, D, INTER, XG, occ, WAVES);
  timeit(name, [&] { hipLaunchKernelGGL((probe_tiled<K, O, NL, NTL, NTS, D, INTER, XG, WAVES>),
                                         dim3(a.total_tiles), dim3(64 * WAVES), lds, 0, a); }, bytes);
}

int main(int argc, char **argv) {
  const char *only = argc > 1 ? argv[1] : "all";
  // same HBM layout as the product bench: shard pitch S + 12 KiB
  g.pitch = kS + 12288;
  CHECK(hipMalloc(&g.data, g.pitch * kShards));
  CHECK(hipMalloc(&g.outp, g.pitch * kShards));
  CHECK(hipMemset(g.data, 0x5a, g.pitch * kShards));
  CHECK(hipMemset(g.outp, 0, g.pitch * kShards));
  CHECK(hipMalloc(&g.d_in, 8 * kShards));
  CHECK(hipMalloc(&g.d_out, 8 * kShards));
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("{\"settle\": \"ok\", \"cus\": %d}\n", cus);
  const bool all = !strcmp(only, "all");
  for (int rep = 0; rep < 2; ++rep) {
    if (all || !strcmp(only, "cal")) {
      // calibration: one read stream, one-stream copy
      run<1, 0, 4, 0, 0, 0, 2, 0>("read");
      run<1, 0, 4, 0, 1, 0, 2, 0>("read");
      run<1, 1, 4, 0, 0, 0, 2, 0>("copy");
      run<1, 1, 4, 0, 0, 1, 2, 0>("copy");
      run<1, 1, 4, 0, 1, 1, 2, 0>("copy");
      run<1, 1, 8, 0, 1, 1, 1, 0>("copy");
      run<1, 1, 2, 0, 1, 1, 4, 0>("copy");
    }
    if (all || !strcmp(only, "rs")) {
      // the product pattern (hc, NL=2, D=2, xg) and the run-length / depth sweep
      run<30, 3, 2, 1, 0, 1, 2, 1>("rs");
      run<30, 0, 2, 1, 0, 1, 2, 1>("rsro");
      run<30, 3, 2, 0, 0, 1, 2, 1>("rs");
      run<30, 3, 4, 0, 0, 1, 2, 1>("rs");
      run<30, 3, 4, 1, 0, 1, 2, 1>("rs");
      run<30, 3, 8, 0, 0, 1, 1, 1>("rs");
      run<30, 3, 8, 0, 0, 1, 2, 1>("rs");
      run<30, 3, 2, 0, 0, 1, 4, 1>("rs");
      run<30, 0, 4, 0, 0, 1, 2, 1>("rsro");
      run<30, 0, 8, 0, 0, 1, 2, 1>("rsro");
      run<30, 3, 4, 0, 1, 1, 2, 1>("rs");
      run<30, 3, 4, 0, 0, 0, 2, 1>("rs");
      run<30, 3, 4, 0, 0, 1, 2, 0>("rs");
    }
    if (all || !strcmp(only, "lds")) {
      run_lds<30, 3, 2, 0, 1, 2>("rs");
      run_lds<30, 3, 4, 0, 1, 2>("rs");
      run_lds<30, 3, 4, 0, 1, 4>("rs");
      run_lds<30, 3, 8, 0, 1, 2>("rs");
      run_lds<30, 3, 4, 1, 1, 2>("rs");
      run_lds<30, 0, 4, 0, 1, 2>("rsro");
      run_lds<1, 1, 4, 0, 1, 2>("copy");
    }
    if (all || !strcmp(only, "occ")) {
      run<30, 3, 2, 1, 0, 1, 2, 1>("rs", 5);  // product v58 pattern at its occupancy
      run<30, 3, 2, 0, 0, 1, 2, 1>("rs", 5);
      run<30, 3, 2, 0, 1, 1, 2, 1>("rs", 5);
      run<30, 3, 2, 0, 1, 1, 2, 1>("rs", 4);
      run<30, 3, 2, 0, 1, 1, 2, 1>("rs", 0);
      run<30, 3, 2, 0, 1, 1, 4, 1>("rs", 5);
      run<30, 3, 2, 0, 1, 0, 2, 1>("rs", 5);
      run<30, 3, 4, 0, 1, 1, 2, 1>("rs", 3);
      run<30, 3, 4, 0, 1, 1, 2, 1>("rs", 4);
      run<30, 3, 4, 0, 1, 1, 1, 1>("rs", 4);
      run<30, 0, 2, 0, 1, 1, 2, 1>("rsro", 5);
      run<8, 3, 2, 0, 1, 1, 2, 1>("rs", 5);
    }
    if (all || !strcmp(only, "pro")) {
      run<30, 3, 2, 0, 1, 1, 2, 1, 0>("rs", 5);
      run<30, 3, 2, 0, 1, 1, 2, 1, 1>("rs", 5);
      run<30, 3, 2, 1, 0, 1, 2, 1, 0>("rs", 5);
      run<30, 3, 2, 1, 0, 1, 2, 1, 1>("rs", 5);
      run<30, 3, 4, 0, 1, 1, 2, 1, 1>("rs", 4);
    }
    if (all || !strcmp(only, "perm")) {
      run<30, 3, 2, 0, 1, 1, 2, 1>("rs", 5);
      run<30, 3, 2, 2, 1, 1, 2, 1>("rs", 5);
      run<30, 0, 2, 0, 1, 1, 2, 1>("rsro", 5);
      run<30, 0, 2, 2, 1, 1, 2, 1>("rsro", 5);
      run<30, 3, 2, 0, 0, 1, 2, 1>("rs", 5);
      run<30, 3, 2, 2, 0, 1, 2, 1>("rs", 5);
    }
    if (all || !strcmp(only, "wg")) {
      // per-wave vs per-workgroup contiguity at the product's settings (ct, nt
      // loads + stores, 3 in flight, XCD grouping, 96-VGPR occupancy)
      run<30, 3, 2, 0, 1, 1, 2, 1, 0, 4>("rs", 5);   // product: 2 KiB/wave, 8 KiB/WG
      run<30, 3, 2, 0, 1, 1, 2, 1, 0, 8>("rs", 5);   // 2 KiB/wave, 16 KiB/WG
      run<30, 3, 4, 0, 1, 1, 2, 1, 0, 4>("rs", 4);   // 4 KiB/wave, 16 KiB/WG
      run<30, 3, 1, 0, 1, 1, 2, 1, 0, 8>("rs", 5);   // 1 KiB/wave, 8 KiB/WG
      run<30, 3, 2, 0, 1, 1, 2, 1, 0, 16>("rs", 5);  // 2 KiB/wave, 32 KiB/WG
    }
    if (!strcmp(only, "ldsplace") && rep == 0) {
      // round 6: the LDS-DMA ring at the occupancy of the
      // computing kernels v107-v109 (tables reserved), beside the register
      // probes, on six separately allocated data sets
      const int copies = 6;
      std::vector<uint8_t *> keep;
      for (int c = 0; c < copies; ++c) {
        uint8_t *d = nullptr;
        CHECK(hipMalloc(&d, g.pitch * kShards));
        CHECK(hipMemset(d, 0x5a, g.pitch * kShards));
        keep.push_back(d);
      }
      for (int c = 0; c < copies; ++c) {
        g.data = keep[c];
        char t[32];
        snprintf(t, sizeof t, "c%d_rs", c);
        run<30, 3, 2, 0, 1, 1, 2, 1, 0, 4>(t, 5);  // product: 2 KiB/wave, registers, 5 waves/SIMD
        run<30, 3, 4, 0, 1, 1, 2, 1, 0, 4>(t, 4);  // 4 KiB/wave, registers
        // probe_lds keeps D+1 slots (its D is the inputs in flight past the
        // consumed one): D=1 -> 2 slots = the kernels' D=2 ring
        run_lds<30, 3, 4, 1, 1, 1, 8>(t, 15360);   // v107: 8 waves, 2 slots: 2 WGs/CU
        run_lds<30, 3, 4, 1, 1, 1, 4>(t, 15360);   // v108: 4 waves, 2 slots: 3 WGs/CU
        run_lds<30, 3, 4, 1, 1, 2, 4>(t, 15360);   // v109: 4 waves, 3 slots: 2 WGs/CU
      }
      return 0;
    }
    if (!strcmp(only, "tplace") && rep == 0) {
      // round 6: row layout (the product's) vs tile-major layout on the same
      // six separately allocated copies; each copy holds the rows at pitch
      // S + 12 KiB (4.03 GB) or the interleaved tiles (4.43 GB)
      const int copies = 6;
      const size_t cbytes = size_t(kShards / 30) * 33 * kS;
      std::vector<uint8_t *> keep;
      for (int c = 0; c < copies; ++c) {
        uint8_t *d = nullptr;
        CHECK(hipMalloc(&d, cbytes));
        CHECK(hipMemset(d, 0x5a, cbytes));
        keep.push_back(d);
      }
      for (int c = 0; c < copies; ++c) {
        g.data = keep[c];
        char t[32];
        snprintf(t, sizeof t, "c%d_rs", c);
        run<30, 3, 2, 0, 1, 1, 2, 1, 0, 4>(t, 5);                  // product rows, 8 KiB/WG
        run_tiled<30, 3, 2, 1, 1, 2, 1, 1>(t, keep[c], g.outp, 5);  // tiles, parity interleaved
        run_tiled<30, 3, 2, 1, 1, 2, 1, 0>(t, keep[c], g.outp, 5);  //   no XCD grouping
        run_tiled<30, 3, 2, 1, 1, 2, 0, 1>(t, keep[c], g.outp, 5);  // tiles, parity separate
        run_tiled<30, 3, 4, 1, 1, 2, 1, 1>(t, keep[c], g.outp, 4);  // 16 KiB tiles
        run_tiled<30, 0, 2, 1, 1, 2, 0, 1>(t, keep[c], g.outp, 5);  // reads only
      }
      return 0;
    }
    if (!strcmp(only, "place") && rep == 0) {
      // placement study: the same patterns on several separately
      // allocated data sets; a pattern whose time does not depend on the copy
      // is robust to where the driver puts the shards
      const int copies = 6;
      std::vector<uint8_t *> keep;
      for (int c = 0; c < copies; ++c) {
        uint8_t *d = nullptr;
        CHECK(hipMalloc(&d, g.pitch * kShards));
        CHECK(hipMemset(d, 0x5a, g.pitch * kShards));
        keep.push_back(d);
      }
      for (int c = 0; c < copies; ++c) {
        g.data = keep[c];
        char t[32];
        snprintf(t, sizeof t, "c%d_rs", c);
        run<30, 3, 2, 0, 1, 1, 2, 1, 0, 4>(t, 5);  // product: 2 KiB/wave, 8 KiB/WG
        run<30, 3, 4, 0, 1, 1, 2, 1, 0, 4>(t, 4);  // 4 KiB/wave
        run<30, 3, 8, 0, 1, 1, 1, 1, 0, 4>(t, 4);  // 8 KiB/wave, 2 in flight
        snprintf(t, sizeof t, "c%d_rsro", c);
        run<30, 0, 2, 0, 1, 1, 2, 1>(t, 5);        // 30 read streams, no writes
        snprintf(t, sizeof t, "c%d_k10", c);
        run<10, 1, 4, 0, 1, 1, 2, 1>(t);
        snprintf(t, sizeof t, "c%d_read", c);
        run<1, 0, 4, 0, 1, 0, 2, 0>(t);
      }
      return 0;
    }
    if (all || !strcmp(only, "mix")) {
      run<10, 1, 4, 0, 0, 1, 2, 1>("mix");
      run<3, 3, 4, 0, 0, 1, 2, 1>("mix");
      run<1, 1, 4, 0, 0, 1, 2, 1>("mix");
    }
  }
  return 0;
}
