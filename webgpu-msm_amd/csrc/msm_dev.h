// Types and constants shared by the HIP kernels (msm_kernels.hip) and their host driver
// (msm_host.cpp).  Internal to libmsm; the public C ABI is include/msm.h.
#pragma once
#include <stdint.h>

namespace msm {

// Geometry of one MSM launch (host fills it, kernels read it by value).
struct MsmDims {
  uint32_t n;      // points
  uint32_t c;      // window bits
  uint32_t B;      // buckets per window = 2^(c-1) (signed digits)
  uint32_t W;      // windows = ceil(257 / c)
  uint32_t fb;     // fine bits sorted inside one coarse bin = min(c-1, 9)
  uint32_t nbc;    // coarse bins per window = B >> fb
  uint32_t nbins;  // W * nbc
  uint32_t ch;     // digits per partition workgroup (one window chunk)
  uint32_t nch;    // chunks per window = ceil(n / ch)
};


constexpr uint32_t PT_WORDS = 36;  // extended point, 4 x 9 limbs (144 B)
constexpr uint32_t PRE_WORDS = 32;  // precomputed affine point record (108 B used, 128 B stride)
constexpr uint32_t KEY_INVALID = 0xffffffffu;
constexpr uint32_t KEY_PASS = 0x80000000u;

constexpr uint32_t MSM_DEV_ERR_COORD_RANGE = 1u;  // a coordinate >= p (bytes.rs:19 panics)
constexpr uint32_t MSM_DEV_ERR_BAD_POINT = 2u;    // z == 0

}  // namespace msm
