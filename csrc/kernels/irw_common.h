// Shared by the fused inverted-residual kernels of two translation units:
// kernels/mbv2_f32.hip (irw_f32, native fp32 MFMA) and kernels/irw_x3.hip
// (irw_x3, split-bf16; built with MFMA results in VGPRs like gemm_x3.hip --
// the 960-hidden 7 x 7 blocks ran 171 -> 156 us with it, the native blocks lost
// up to 8 %: profiles/r5_vgpr_form_ab.txt).  Tile geometry, the in-launch
// combine of hidden parts, and the configuration record.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "kernels/gemm_f32.h"
#include "kernels/mbv2.h"
#include "kernels/x3.h"

namespace nnsx {
namespace kernels {

// wave-split kernel configurations: the 28x28 / 14x14 / 7x7 blocks of MobileNetV2
struct IrwCfg {
  int S, TY, TX, KIN, NOT, NW;
  bool full;
  void (*kernel)(IrBlockF32Args);
  size_t (*lds)(int);
  int dil = 1;
  // > 0: only for exactly tiled maps and batches >= min_batch (find_irw with the
  // launch's batch; a support query without one never picks it)
  int min_batch = 0;
  // > 0: only for batches <= max_batch (a support query must name its batch)
  int max_batch = 0;
};

// the x3 twins of the fused-block configurations (kernels/irw_x3.hip)
const std::vector<IrwCfg>& x3_irw_cfgs();
// 14 x 14 blocks, one image per workgroup, split-bf16 (kernels/irp_x3.hip);
// needs a.we3 / a.wp3.  false: not this shape (or NNSX_IRP=0)
bool irp_x3_supported(const IrBlockF32Args& a);
bool irp_x3(const IrBlockF32Args& a, hipStream_t s);
// smallest batch the image-per-workgroup kernels take (default 128, NNSX_IRP_MIN_B); returns the old value
int irp_x3_set_min_batch(int b);
// the 28 x 28 half-image kernels (kernels/irp_x3.hip): 0 off, 1 stride 2, 2 both; returns the old mode
int irh_set_mode(int m);

namespace {

template <int S, int TY, int TX, int KIN, int NOT, int NW, bool FULL, int DIL = 1>
struct IrwGeom {
  static constexpr int TIY = (TY - 1) * S + 2 * DIL + 1, TIX = (TX - 1) * S + 2 * DIL + 1;
  static constexpr int PIN = TIY * TIX;               // halo grid cells
  static constexpr int NC16 = (PIN + 15) / 16 * 16;   // compact in-image pixels (max), padded
  static constexpr int NBT = NC16 / 16;               // expand pixel tiles
  // LDS planes are multiples of 256 B (16 quads): a ds_read_b128 lane group
  // ({0-3,12-15} of one 16-lane half + {4-11} of the next, etc.) then hits
  // disjoint bank slots when each half reads 16 consecutive quads of its own
  // plane.  xs positions are XOR-swizzled with (kq & 3) so the staging writes
  // (8 consecutive lanes = 8 k-quads of one pixel) land in 4 slots, not 1.
  static constexpr int XSP = NC16;                    // xs plane stride (quads)
  // hidden plane stride (quads); the compact expand (FULL = false) needs one
  // scratch cell past the grid for padding pixels
  static constexpr int PINP = FULL ? (PIN + 15) / 16 * 16 : PIN / 16 * 16 + 16;
  static constexpr int KQ = KIN / 4;
  static constexpr int NPT = (TY * TX + 15) / 16;     // output pixel tiles
  static constexpr int NPX = NPT * 16;
  static constexpr size_t xs_q = static_cast<size_t>(KQ) * XSP;
  static constexpr size_t hid_q = static_cast<size_t>(4 * NW) * PINP;     // [wave][quad][cell]
  static constexpr size_t red_q = static_cast<size_t>(2 * 4 * NW) * NPX;  // [buf][wave][quad][px]
  static size_t lds_bytes(int) { return 16 * std::max(xs_q + hid_q, red_q); }
  // minimum waves per SIMD the register budget is sized for (hipcc reads the
  // second launch bound that way).  4 (128 VGPRs) where the LDS allows more
  // workgroups than the registers: 28x28 (KIN 32) measured 57 -> 53.5 us at
  // batch 128 despite 6 spilled VGPRs; the same on the 14x14 64-channel block
  // (3, 21 spills) lost 40 -> 45 us, and on the 56x56 block (1 spill, 5
  // workgroups/CU instead of 4) 128 -> 144 us.
  // (the wider 7x14 28x28 tiles hold 14 accumulators: 3 waves per SIMD)
  // (7x14 tiles with 6 cout tiles: 42 accumulators; the LDS holds one workgroup
  // per CU anyway, so one wave per SIMD and the accumulation registers)
  // (5 x 15 tiles on 24 channels: 170 VGPRs at 2, two waves per SIMD where the LDS
  // holds three)
  static constexpr int MINB = (KIN == 32 && S == 1) ? (TY * TX <= 49 ? 4 : 3)
                              : (KIN == 24 && S == 1 && TY == 5) ? 3
                              : (NOT <= 4 || (NOT <= 6 && TY * TX <= 64)) ? 2 : 1;
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// In-launch combine of a tile's hidden parts (irw_f32 / irw_x3), after every
// part wrote its slab write-through (sc1) to a.ws.
template <int TY, int TX, int NT>
__device__ __forceinline__ void irw_inlaunch_combine(const IrBlockF32Args& a, float* smem, int tile, int part,
                                                     int nparts, int b, int oy0, int ox0, int tid) {
  // ---- in-launch combine of the hidden parts (MI355X hand-off, counter form):
  // every part's slab went out write-through (sc1, so no release fence); each
  // storing wave drains it, the workgroup meets at a barrier, one lane draws a
  // ticket; the tile's last part reads every slab with sc1 loads (so no acquire
  // fence either) and adds them in part order, + bias (+ residual) -- the sums
  // of irw_reduce in its order, without its launch -- then resets the ticket
  // for the next launch (tickets start at zero: the caller's buffer is zeroed
  // once at creation).  Correct for any placement of the parts over XCDs.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's slab stores done; the LDS is free
  const int64_t plane = static_cast<int64_t>(a.B) * a.Ho * a.Wo * a.cout;
  const __amdgpu_buffer_rsrc_t slab =
      __builtin_amdgcn_make_buffer_rsrc(a.ws, 0, static_cast<int>(nparts * plane * sizeof(float)), 0x00020000);
  const int nq = a.cout / 4;
  // the tile's output quads [v0, v1): all of them (last-arriver form) or this
  // part's share (spread form), summed over the slabs in part order
  auto combine = [&](int v0, int v1) {
    for (int v = v0 + tid; v < v1; v += NT) {
      const int q = v / nq, co = (v - q * nq) * 4;
      const int gy = oy0 + q / TX, gx = ox0 + q % TX;
      if (gy >= a.Ho || gx >= a.Wo) continue;
      const int64_t e = ((static_cast<int64_t>(b) * a.Ho + gy) * a.Wo + gx) * a.cout + co;
      f32x4_t s =
          __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(slab, static_cast<int>(e * 4), 0, 16));
      for (int p = 1; p < nparts; ++p)
        s += __builtin_bit_cast(
            f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(slab, static_cast<int>((p * plane + e) * 4), 0, 16));
      s += *reinterpret_cast<const f32x4_t*>(a.bp + co);
      if (a.residual) s += *reinterpret_cast<const f32x4_t*>(a.x + (e / a.cout) * a.cin + co);
      *reinterpret_cast<f32x4_t*>(a.y + e) = s;
    }
  };
  if (a.spread) {
    // spread form: one lane per part bumps the tile's monotone 64-bit arrival
    // count and waits until every part of this launch has arrived (count >=
    // the next multiple of nparts); then each part adds its 1/nparts share.
    // The host launches this form only when the whole grid is resident at
    // once; the wait is bounded all the same (~0.2 s), so a broken residency
    // assumption shows up as wrong sums, never as a hung GPU.
    if (tid == 0) {
      unsigned long long* ctr = reinterpret_cast<unsigned long long*>(a.tickets) + tile;
      const unsigned long long t = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long target = (t / nparts + 1) * nparts;
      for (int it = 0; it < (1 << 21); ++it) {
        if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the wait)
    const int total = TY * TX * nq, chunk = (total + nparts - 1) / nparts;
    combine(part * chunk, min(total, (part + 1) * chunk));
    return;
  }
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(a.tickets + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == nparts - 1;
    if (last) __hip_atomic_store(a.tickets + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the ticket)
  combine(0, TY * TX * nq);
}


}  // namespace
}  // namespace kernels
}  // namespace nnsx
