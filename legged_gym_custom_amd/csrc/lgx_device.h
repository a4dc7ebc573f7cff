// lgx_device.h — small device helpers for the env-step kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LGX_DEV __device__ __forceinline__

// ---------------------------------------------------------------- wave helpers
template <int CTRL>
LGX_DEV float dpp_shr_t(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}

// Sum over lanes 0..15 (DPP row 0), returned to every lane. Lanes 0..15 must be active;
// the other rows' values are ignored.
LGX_DEV float row0_sum16(float x) {
  x += dpp_shr_t<0x111>(x);
  x += dpp_shr_t<0x112>(x);
  x += dpp_shr_t<0x114>(x);
  x += dpp_shr_t<0x118>(x);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 15));
}

LGX_DEV int lane_id() { return __lane_id(); }

// ---------------------------------------------------------------- Philox4x32-10
// Same definition as oracle/philox.py and oracle/lgx_oracle.c (counter layout:
// c0 = global env id, c1/c3 = step lo/hi, c2 = block | stream << 16; key = seed).
LGX_DEV void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                           uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
LGX_DEV float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// ---------------------------------------------------------------- fp32 vector math
struct f3 {
  float x, y, z;
};
LGX_DEV f3 mk(float x, float y, float z) { return f3{x, y, z}; }
LGX_DEV f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
LGX_DEV void st3(float* p, f3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
LGX_DEV f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
LGX_DEV f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
LGX_DEV f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
LGX_DEV float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
LGX_DEV f3 cross(f3 a, f3 b) { return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
// row-major 3x3
LGX_DEV f3 mv(const float* R, f3 v) {
  return f3{R[0] * v.x + R[1] * v.y + R[2] * v.z, R[3] * v.x + R[4] * v.y + R[5] * v.z,
            R[6] * v.x + R[7] * v.y + R[8] * v.z};
}
LGX_DEV void mm(const float* A, const float* B, float* O) {
  float T[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) T[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
#pragma unroll
  for (int i = 0; i < 9; ++i) O[i] = T[i];
}
// symmetric inertia (xx yy zz xy xz yz) times vector
LGX_DEV f3 symv(const float* I, f3 v) {
  return f3{I[0] * v.x + I[3] * v.y + I[4] * v.z, I[3] * v.x + I[1] * v.y + I[5] * v.z,
            I[4] * v.x + I[5] * v.y + I[2] * v.z};
}
LGX_DEV void quat_to_R(const float* q, float* R) {
  float x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}
