// Types and constants shared by the HIP kernels (msm_kernels.hip) and their host driver
// (msm_host.cpp).  Internal to libmsm; the public C ABI is include/msm.h.
#pragma once
#include <stdint.h>

namespace msm {

// Geometry of one MSM launch (host fills it, kernels read it by value).
// Windows (balanced widths): W - 1 "main" windows cover scalar bits [0, 254) -- the first nhi of
// them q + 1 bits wide, the rest q bits -- and one 3-bit overflow window covers bits [254, 256)
// plus the carry.  A scalar < 2^253 (any canonical Fr/Fq value) never carries out of the top main
// window, so the overflow window only holds digits of non-canonical 256-bit scalars.  Balancing
// keeps the top main window as wide as the others (a ragged top window of a few bits would turn
// into a handful of giant buckets).
// A launch may carry a BATCH of nm independent MSMs of n points each (small MSMs fill the machine
// together): MSM m owns windows [m Wm, (m+1) Wm) and point records [m n, (m+1) n); every kernel
// after the recode sees W = nm Wm windows and does not care which MSM a window belongs to.
constexpr uint32_t MSM_MAX_BATCH = 8;
struct BatchPtrs {  // per-MSM input buffers of a batch (kernel argument, by value)
  const uint32_t* p[MSM_MAX_BATCH];
};
struct MsmDims {
  uint32_t n;      // points per MSM
  uint32_t c;      // widest window (bits); digit codes and bucket tables are sized for it
  uint32_t B;      // buckets per window = 2^(c-1) (signed digits; narrower windows use fewer)
  uint32_t W;      // windows of the whole batch = nm * Wr
  uint32_t Wm;     // windows per MSM, overflow window included (all of them are recoded)
  uint32_t w0;     // window range of this launch (msm_opts MSM_FLAG_WINDOWS): windows
  uint32_t Wr;     //   [w0, w0 + Wr) of every MSM; local window l of an MSM is window w0 + l
  uint32_t half_lo;  // MSM_FLAG_HALF_WINDOWS: local window 0 keeps only its upper-half buckets,
  uint32_t half_hi;  //   local window Wr - 1 only its lower-half buckets (digit magnitudes)
  uint32_t nm;     // MSMs in the batch
  uint32_t q;      // main-window base width
  uint32_t nhi;    // main windows of width q + 1
  uint32_t fb;     // fine bits sorted inside one coarse bin = min(c-1, 9)
  uint32_t nbc;    // coarse bins per window = B >> fb
  uint32_t nbins;  // W * nbc
  uint32_t ch;     // digits per partition workgroup (one window chunk)
  uint32_t nch;    // chunks per window = ceil(n / ch)
  uint32_t packed; // coarse-binned entries carry their fine key: (entry << fb) | fine in one u32
                   // (when nm n <= 2^(31 - fb)); else a separate u16 array holds the fine keys
  uint32_t shared; // every MSM of the batch uses ONE base vector (prover batch): entries index
                   // point records [0, n) instead of [m n, (m+1) n)
};


constexpr uint32_t MAIN_BITS = 254;  // bits covered by the main windows (scalars < 2^253, + carry)
constexpr uint32_t OVF_BITS = 3;     // overflow window: bits 254, 255 and the carry (digit <= 4)

// Width and bit offset of window w (w < Wm: a window of one MSM, counted from the least
// significant; a launch's local window l is window d.w0 + l).
__host__ __device__ inline uint32_t win_bits(const MsmDims& d, uint32_t w) {
  return w + 1 == d.Wm ? OVF_BITS : (w < d.nhi ? d.q + 1 : d.q);
}
__host__ __device__ inline uint32_t win_off(const MsmDims& d, uint32_t w) {
  return w * d.q + (w < d.nhi ? w : d.nhi);
}

constexpr uint32_t PT_WORDS = 36;  // extended point, 4 x 9 limbs (144 B)
// Precomputed affine point record, 128 B (one cache line), in two 48-B halves the gather can swap:
//   words  0..8  (y-x)/2   9 d*t limb 8   10 (y+x)/2 limb 8   11 zero
//   words 12..20 (y+x)/2  21 d*t limb 8   22 (y-x)/2 limb 8   23 zero
//   words 24..31 d*t limbs 0..7
// A negated point (-x, y) swaps (y-x)/2 and (y+x)/2: k_accumulate reads the half at PRE_HALF * sign
// first, so the swap is an address offset, not 18 selects (load_pre_signed).  The half read first
// (12 words) holds every top limb, so the other half costs only its 8 low words: 7 loads.
constexpr uint32_t PRE_WORDS = 32;
constexpr uint32_t PRE_HALF = 12;  // words per swappable half
constexpr uint32_t PRE_KT = 24;    // d*t limbs 0..7
constexpr uint32_t KEY_INVALID = 0xffffffffu;
constexpr uint32_t KEY_PASS = 0x80000000u;

constexpr uint32_t MSM_DEV_ERR_COORD_RANGE = 1u;  // a coordinate >= p (bytes.rs:19 panics)
constexpr uint32_t MSM_DEV_ERR_BAD_POINT = 2u;    // z == 0

}  // namespace msm
