// MFMA shape vs sustained rate under the power limit (round 6 experiment, not product code).
// Each wave computes a 64x64 fp32 tile with the S8 3 x bf16 products, K step 32, its operands read
// from LDS (16 x 16-byte reads per step per wave, the same for both shapes), at 2 blocks of 4 waves
// per CU (the update's GEMM occupancy). Shape 16: v_mfma_f32_16x16x32_bf16 (48 per step);
// shape 32: v_mfma_f32_32x32x16_bf16 (24 per step, the same flops). Reports TF/s (bf16 products)
// and the shader clock (s_memtime cycles over s_memrealtime ticks at 100 MHz).
// data 0: hi/lo of N(0,1) values; 1: lo planes zero; 2: everything zero.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/exp/mfma_power tools/exp/mfma_power.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <random>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define LDS_BYTES 65536

template <int SHAPE, int ORDER>
__global__ __launch_bounds__(256, 2) void mfma_loop(const uint4* __restrict__ src, float* __restrict__ out,
                                                    unsigned long long* __restrict__ clk, int iters) {
  extern __shared__ uint4 lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < LDS_BYTES / 16; i += 256) lds[i] = src[(blockIdx.x * 97 + i) % (LDS_BYTES / 16 * 4)];
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  // 4 waves, each reads its own 16 KB quarter; 16 reads of 64 lanes x 16 B = 16 KB per step
  const uint4* base = lds + w * 1024;
  if constexpr (SHAPE == 16 || SHAPE == 0) {
    f32x4 acc[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    bf16x8 ah[4], al[4], bh[4], bl[4];
    for (int it = 0; it < iters; ++it) {
      const int o = (it & 1) * 64;
#pragma unroll
      for (int i = 0; i < 4 && (SHAPE == 16 || it == 0); ++i) {
        uint4 x = base[(i * 4 + 0) * 64 + lane ^ o];
        uint4 y = base[(i * 4 + 1) * 64 + lane ^ o];
        uint4 z = base[(i * 4 + 2) * 64 + lane ^ o];
        uint4 v = base[(i * 4 + 3) * 64 + lane ^ o];
        memcpy(&ah[i], &x, 16); memcpy(&al[i], &y, 16); memcpy(&bh[i], &z, 16); memcpy(&bl[i], &v, 16);
      }
      if constexpr (ORDER == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
      } else {
        // grouped by product: one operand register set held over 4 consecutive MFMAs
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
      }
    }
    float s = 0;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 256 + tid] = s;
  } else {
    f32x16 acc[2][2];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
    for (int it = 0; it < iters; ++it) {
      const int o = (it & 1) * 64;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          uint4 x = base[(ks * 8 + i * 4 + 0) * 64 + lane ^ o];
          uint4 y = base[(ks * 8 + i * 4 + 1) * 64 + lane ^ o];
          uint4 z = base[(ks * 8 + i * 4 + 2) * 64 + lane ^ o];
          uint4 v = base[(ks * 8 + i * 4 + 3) * 64 + lane ^ o];
          memcpy(&ah[i], &x, 16); memcpy(&al[i], &y, 16); memcpy(&bh[i], &z, 16); memcpy(&bl[i], &v, 16);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
    }
    float s = 0;
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int r = 0; r < 16; ++r) s += acc[i][j][r];
    out[blockIdx.x * 256 + tid] = s;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    clk[(blockIdx.x * 4 + w) * 2 + 0] = t1 - t0;
    clk[(blockIdx.x * 4 + w) * 2 + 1] = r1 - r0;
  }
}

static unsigned short bf16_bits(float x) {  // round to nearest even
  unsigned u;
  memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
static float bf16_val(unsigned short h) {
  unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 512, iters = argc > 2 ? atoi(argv[2]) : 256;
  const size_t n16 = LDS_BYTES / 16 * 4;  // uint4 elements of the source
  std::vector<unsigned short> h(n16 * 8);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd;
  for (size_t i = 0; i < h.size(); i += 16) {  // 8 hi then 8 lo of the same 8 values (one 32-B S8 group)
    for (int k = 0; k < 8; ++k) {
      float x = nd(rng);
      unsigned short hi = bf16_bits(x);
      h[i + k] = hi;
      h[i + 8 + k] = bf16_bits(x - bf16_val(hi));
    }
  }
  uint4 *d_src[3];
  for (int d = 0; d < 3; ++d) {
    std::vector<unsigned short> v = h;
    if (d >= 1)
      for (size_t i = 0; i < v.size(); i += 16)
        for (int k = 0; k < 8; ++k) v[i + 8 + k] = 0;
    if (d == 2) std::fill(v.begin(), v.end(), 0);
    CK(hipMalloc(&d_src[d], n16 * 16));
    CK(hipMemcpy(d_src[d], v.data(), n16 * 16, hipMemcpyHostToDevice));
  }
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, blocks * 256 * 4));
  CK(hipMalloc(&clk, blocks * 4 * 2 * 8));
  std::vector<unsigned long long> hc(blocks * 8);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int v : {0, 100, 16, 116, 32}) {
    const int shape = v % 100, order = v / 100;
    for (int d = 0; d < 3; ++d) {
      auto launch = [&]() {
        if (v == 0)
          mfma_loop<0, 0><<<blocks, 256, LDS_BYTES>>>(d_src[d], out, clk, iters);
        else if (v == 100)
          mfma_loop<0, 1><<<blocks, 256, LDS_BYTES>>>(d_src[d], out, clk, iters);
        else if (v == 16)
          mfma_loop<16, 0><<<blocks, 256, LDS_BYTES>>>(d_src[d], out, clk, iters);
        else if (v == 116)
          mfma_loop<16, 1><<<blocks, 256, LDS_BYTES>>>(d_src[d], out, clk, iters);
        else
          mfma_loop<32, 0><<<blocks, 256, LDS_BYTES>>>(d_src[d], out, clk, iters);
      };
      launch();
      launch();
      CK(hipDeviceSynchronize());
      const int reps = 5;
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(hc.data(), clk, hc.size() * 8, hipMemcpyDeviceToHost));
      double cyc = 0, rt = 0;
      for (int i = 0; i < blocks * 4; ++i) cyc += hc[2 * i], rt += hc[2 * i + 1];
      double flops = double(blocks) * 4 * iters * 48 * 16384.0 * reps;
      printf("shape %d order %d (shape 0: 16x16 operands in registers; order 1: grouped by product) data %d: %.3f ms/launch  %.1f TF/s (bf16 products)  clock %.0f MHz\n", shape, order, d,
             ms / reps, flops / (ms * 1e-3) / 1e12, cyc / rt * 100.0);
    }
  }
  return 0;
}
