// Implicit-GEMM conv2d for gfx950 (MFMA), NHWC activations — forward, backward-data and
// backward-weight of the convolutions in ResNetSQ (torchvision resnet18 via
// torch/models.py:181-184) and GenericNetSQ (torch/models.py:134-152).
//
// Two kernel families, both 256 threads = 4 wave64, LDS double-buffered, register-staged
// 16-byte global loads, fp32 accumulation:
//
//   conv_nt_kernel  (forward, backward-data): out[m][n] = sum_k Q[m][k] * P[n][k]
//       Q = implicit im2col of an NHWC tensor (X for fwd, dY for dgrad), k = (tap, channel),
//           gathered on the fly (src pixel = o*ms + off + tap*ks, zero outside); a strided
//           dgrad runs as stride*stride parity classes, each a stride-1 gather over dY with only
//           the taps of that class (no multiplications by structural zeros);
//       P = packed weights, k-contiguous ([K][R][S][C] fwd, [C][R][S][K] dgrad).
//       LDS rows are 128 B (64 bf16 / 32 f32 of k) with a 16-B-slot XOR swizzle
//       slot ^= (row>>1)&7 that makes the ds_read_b128 fragment reads conflict-free.
//   conv_tn_kernel  (backward-weight): dW[kout][(tap,c)] = sum_pixels dY[p][kout] * X~[p][(tap,c)]
//       Both operands are pixel-major (k-outer), staged as [k][col] LDS tiles and read into MFMA
//       fragments with the gfx950 transposing LDS read ds_read_b64_tr_b16 (bf16).  The pixel
//       dimension (N*Ho*Wo, up to 1M) is split across workgroups (split-K) into fp32 slabs that a
//       reduce kernel sums in a fixed order (bitwise reproducible) while permuting to torch's
//       [K][C][R][S] weight-grad layout.
//
// MFMA: bf16 / fp16 -> v_mfma_f32_16x16x32_{bf16,f16}; f32 (parity mode) -> v_mfma_f32_16x16x4_f32 (exact
// f32 products, f32 accumulation).  The MFMA A operand is always the output's contiguous
// dimension, so each lane owns 4 consecutive output channels of one pixel and stores them with
// one 8-B (bf16) / 16-B (f32) store — no LDS epilogue.
// Convs whose input has < 8 channels (conv1: C=1) run as an explicit im2col (K padded to 64) +
// 1x1 GEMM through the same kernels.
#include <stdint.h>
#include <stdlib.h>
#include "sqr_conv_dev.h"
#include "sqr_bn_dev.h"

namespace sqr {
namespace conv {

// implicit im2col view of an NHWC tensor
struct Gather {
  const void* base;
  int Hi, Wi, Ci, log2Ci;  // source tensor [N][Hi][Wi][Ci]
  int Ho, Wo;              // pixel grid of the GEMM rows
  int ms, off_h, off_w, ks; // src = o*ms + off + r*ks
  int R, S;
  int M;                   // N*Ho*Wo
  FastDiv fd_hw, fd_w;     // divide by Ho*Wo, Wo
  FastDiv fd_s;            // divide by S (tap -> r, s)
  uint32_t bytes;          // size of the source tensor (buffer-descriptor range)
};

struct NTArgs {
  Gather g;        // Q operand  [M][Kg]
  const void* w;   // P operand  [Nout][Kg]
  int Nout, Kg;    // Kg = R*S*Ci (multiple of 8)
  void* out;       // [M][Nout] (os == 1) or the strided pixel subset of an [N][oH][oW][Nout] tensor
  int os, oph, opw, oH, oW;  // out pixel of row (n,i,j) = (n, i*os+oph, j*os+opw)
  int ntm, ntn;    // tile counts
  float* stats;    // nullable: per-M-tile BatchNorm Welford rows [ntm][2][Nout] (mean, M2) + [ntm] counts
};

// up to 4 independent NT GEMMs in one launch (the stride-parity classes of a strided dgrad):
// blocks [start[i], start[i+1]) of the XCD-remapped id space run class i
struct NTMulti {
  NTArgs c[4];
  int start[4];
  int ncls;
  unsigned long long* tp;  // nullable: clock probe slots
};

struct TNArgs {
  Gather g;          // P operand: X gathered, [pixels][Ng], Ng = R*S*Ci
  const void* dy;    // Q operand: dY [pixels][Kout]
  int Kout, Ng;
  int kchunk;        // pixels per split
  float* slab;       // [splits][Kout][Ng]
  int ntm, ntn;
  int rect_wt;       // > 0: every BK-pixel tile is a rect_wt-wide rectangle of one image (no divides)
  unsigned long long* tp;  // nullable: clock probe slots
};

// ============================================================================ NT (fwd / dgrad)
// 16-B zero source for LDS-DMA lanes whose im2col element lies in the padding
__device__ __attribute__((aligned(64))) unsigned int g_zero16[16];

__device__ __forceinline__ void glds16(const void* src, char* lds_row_block) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_row_block, 16, 0, 0);
}

// STAGES-deep LDS ring filled by global_load_lds_dwordx4 (LDS-DMA: no staging registers, no
// ds_write).  One wave-instruction writes 1 KiB = 8 LDS rows x 8 slots; lane l lands in physical
// slot l&7 of row l>>3, so each lane loads the LOGICAL slot (l&7) ^ swz(row) — the XOR swizzle is
// applied on the source address (rule: linear LDS destination, inverse-swizzled source).  Loads of
// tiles kt+1..kt+STAGES-1 stay in flight across the raw s_barrier; a counted s_waitcnt vmcnt
// retires exactly the tile read next.
template <typename T, int BM, int BN, int WAVES_M, int WAVES_N, int STAGES>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N) conv_nt_kernel(NTMulti mc) {
  using C = Cfg<T>;
  constexpr int BK = 128 / C::ES;  // k elements per LDS row (128 B)
  constexpr int ROWB = 128;
  constexpr int NW = WAVES_M * WAVES_N, NT = 64 * NW;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int QV = BM / (8 * NW), PV = BN / (8 * NW);  // glds per wave per tile for Q / P
  constexpr int PER_TILE = QV + PV;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(QV >= 1 && PV >= 1 && QV * 8 * NW == BM && PV * 8 * NW == BN, "tile rows per wave");
  constexpr int TILE_Q = BM * ROWB, TILE_P = BN * ROWB, STAGE = TILE_Q + TILE_P;
  // ONE __shared__ array, no other LDS reads in the loop: an LDS read that may alias an in-flight
  // LDS-DMA makes hipcc insert s_waitcnt vmcnt(0) in front of it (that killed the pipeline when
  // the tap table lived in LDS) — tap -> (r, s) is computed with a multiply-high instead.
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];
  clock_begin(mc.tp);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bid_all = xcd_remap(blockIdx.x, gridDim.x);
  const int cls = mc.ncls == 1 ? 0
                               : (int)(bid_all >= mc.start[1]) + (int)(mc.ncls > 2 && bid_all >= mc.start[2]) +
                                     (int)(mc.ncls > 3 && bid_all >= mc.start[3]);
  const NTArgs& a = mc.c[cls];
  const int bid = bid_all - mc.start[cls];
  const Gather& g = a.g;
  const int tile_m = bid / a.ntn, tile_n = bid % a.ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // this lane's rows: r_i = 8*(NW*i + wave) + (lane>>3); its logical slot is the same for every i
  // (NW even: the row swizzle (r>>1)&7 = (4*wave + (lane>>4))&7).
  // Loads go through buffer descriptors: an out-of-range voffset returns zeros, so padding /
  // out-of-tensor lanes just get voffset = kOOB and the per-row work is a few 32-bit VALU ops.
  constexpr uint32_t kOOB = 0x80000000u;
  const int lrow = lane >> 3;
  const int lslot = (lane & 7) ^ ((4 * wave + (lane >> 4)) & 7);
  int q_off[QV], q_hb[QV], q_wb[QV];
#pragma unroll
  for (int i = 0; i < QV; ++i) {
    const int m = m0 + 8 * (NW * i + wave) + lrow;
    if (m < g.M) {
      const int n = (int)fdiv((uint32_t)m, g.fd_hw);
      const int rem = m - n * g.Ho * g.Wo;
      const int oh = (int)fdiv((uint32_t)rem, g.fd_w);
      const int ow = rem - oh * g.Wo;
      q_hb[i] = oh * g.ms + g.off_h;
      q_wb[i] = ow * g.ms + g.off_w;
      q_off[i] = ((n * g.Hi + q_hb[i]) * g.Wi + q_wb[i]) * g.Ci * C::ES;  // may be < 0 (padding)
    } else {
      q_hb[i] = q_wb[i] = -(1 << 28);  // fails every bounds test
      q_off[i] = 0;
    }
  }
  uint32_t p_off[PV];
#pragma unroll
  for (int i = 0; i < PV; ++i) {
    const int n = n0 + 8 * (NW * i + wave) + lrow;
    p_off[i] = n < a.Nout ? (uint32_t)(n * a.Kg * C::ES) : kOOB;
  }
  const __amdgpu_buffer_rsrc_t qsrd = __builtin_amdgcn_make_buffer_rsrc((void*)g.base, 0, g.bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t psrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, (uint32_t)(a.Nout * a.Kg * C::ES), 0x00020000);
  const int RS = g.R * g.S;
  const int nkt = (a.Kg + BK - 1) / BK;
  // the loop's scalars as locals: read through `a`/`g` (a dynamically indexed kernel argument) they
  // were re-loaded with s_load + s_waitcnt lgkmcnt(0) in every k step (the asm "memory" clobbers)
  const int gHi = g.Hi, gWi = g.Wi, gCi = g.Ci, glog2Ci = g.log2Ci, gS = g.S, gks = g.ks, Kg = a.Kg;
  const FastDiv fds = g.fd_s;

  auto issue = [&](int kt, int stage) {
    char* q = smem + stage * STAGE;
    char* p = q + TILE_Q;
    const int k = kt * BK + lslot * C::VEC;
    const int tap = k >> glog2Ci;
    const int c = k & (gCi - 1);
    const bool tap_ok = tap < RS;
    const int tr = (int)fdiv((uint32_t)tap, fds);
    const int dh = tr * gks, dw = (tap - tr * gS) * gks;
    const int tapoff = ((dh * gWi + dw) * gCi + c) * C::ES;
#pragma unroll
    for (int i = 0; i < QV; ++i) {
      const int h = q_hb[i] + dh, w = q_wb[i] + dw;
      const bool ok = tap_ok && (unsigned)h < (unsigned)gHi && (unsigned)w < (unsigned)gWi;
      const uint32_t voff = ok ? (uint32_t)(q_off[i] + tapoff) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qsrd, (__attribute__((address_space(3))) void*)(q + (8 * (NW * i + wave)) * ROWB),
                                               16, voff, 0, 0, 0);
    }
    const uint32_t kb = (uint32_t)(k * C::ES);
    const bool k_ok = k < Kg;
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const uint32_t voff = k_ok ? p_off[i] + kb : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(psrd, (__attribute__((address_space(3))) void*)(p + (8 * (NW * i + wave)) * ROWB),
                                               16, voff, 0, 0, 0);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nkt) issue(s, s);
  if (nkt >= STAGES - 1) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_TILE * (STAGES - 2)) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt % STAGES;
    const bool more = kt + STAGES - 1 < nkt;
    if (more) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const char* q = smem + cur * STAGE;
    const char* p = q + TILE_Q;
#pragma unroll
    for (int sub = 0; sub < BK / C::KSUB; ++sub) {
      if constexpr (C::ES == 2) {
        V8<T> pf[TN], qf[TM];
        const int slot = 4 * sub + fq;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * WN + 16 * j + fr;
          pf[j] = *(const V8<T>*)(p + row * ROWB + nt_swz(row, slot) * 16);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + 16 * i + fr;
          qf[i] = *(const V8<T>*)(q + row * ROWB + nt_swz(row, slot) * 16);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
      } else {
        float pf[TN], qf[TM];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * WN + 16 * j + fr;
          pf[j] = *(const float*)(p + row * ROWB + nt_swz(row, sub) * 16 + fq * 4);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + 16 * i + fr;
          qf[i] = *(const float*)(q + row * ROWB + nt_swz(row, sub) * 16 + fq * 4);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
      }
    }
    // retire tile kt+1 (leave the younger tiles in flight), then let every wave see it; lgkmcnt(0):
    // this wave's reads of tile kt are done before the barrier after which tile kt's stage is refilled
    if (more) {
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_TILE * (STAGES - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: lane holds out[m][n..n+3]
  T* __restrict__ out = (T*)a.out;
  size_t orow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * WM + 16 * i + fr;
    if (a.os == 1) {
      orow[i] = (size_t)m;
    } else {
      const int n = (int)fdiv((uint32_t)m, g.fd_hw);
      const int rem = m - n * g.Ho * g.Wo;
      const int oi = (int)fdiv((uint32_t)rem, g.fd_w);
      const int oj = rem - oi * g.Wo;
      orow[i] = ((size_t)n * a.oH + oi * a.os + a.oph) * a.oW + oj * a.os + a.opw;
    }
  }
  bool wide = false;
  if constexpr (C::ES == 2 && TN % 2 == 0) wide = a.Nout % 8 == 0;
  if constexpr (C::ES == 2 && TN % 2 == 0) {
    if (wide) {
      // 16-bit output in 16-B stores: v_permlane16_swap of tile pair (j, j+1) leaves lane (fr, fq)
      // the 8 contiguous channels 16 (j + (fq & 1)) + 8 (fq >> 1) .. +7 of its pixel (as in the
      // direct 3x3 kernels' epilogue: half the store instructions, same bytes)
      const int sw = 12 * (fq & 1);
#pragma unroll
      for (int j = 0; j + 1 < TN; j += 2) {
        const int n = n0 + wn * WN + 16 * j + 4 * fq + sw;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const auto r0 = __builtin_amdgcn_permlane16_swap(pack2<T>(acc[j][i][0], acc[j][i][1]),
                                                           pack2<T>(acc[j + 1][i][0], acc[j + 1][i][1]), false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(pack2<T>(acc[j][i][2], acc[j][i][3]),
                                                           pack2<T>(acc[j + 1][i][2], acc[j + 1][i][3]), false, false);
          const int m = m0 + wm * WM + 16 * i + fr;
          if (m < g.M && n < a.Nout) *(u32x4*)(out + orow[i] * a.Nout + n) = u32x4{r0[0], r1[0], r0[1], r1[1]};
        }
      }
    }
  }
  if (!wide) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + 16 * j + 4 * fq;
      if (n >= a.Nout) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * WM + 16 * i + fr;
        if (m < g.M) store4(out + orow[i] * a.Nout + n, acc[j][i]);
      }
    }
  }
  if (a.stats) {
    // fused BatchNorm statistics of the STORED (dtype-rounded) output: this M-tile's Welford row
    // (mean, M2) per channel -> stats[tile_m][0/1][n] and its pixel count after the ntm rows (the BN
    // layer finalizes from these partials instead of re-reading the whole activation).  The 16 lanes
    // of a quarter-wave (same fq: the same 4 channels, 16 pixels per i) shift by the group's first
    // value K (lane fr = 0, i = 0: the group's smallest pixel, valid whenever any of its pixels is),
    // add their shifted values / squares / counts as plain floats over an xor tree (no division per
    // level), and the group rows (n, mean = K + S/n, M2 = Q - S^2/n) of the WAVES_M wave rows are
    // merged per column in a fixed order with Chan's formula (counts differ in a partial last tile).
    float* red = (float*)smem;  // [WAVES_M][BN][3]; the k loop ended with a barrier
    auto chan = [](float& n, float& m, float& q, float nb, float mb, float qb) {
      const float nn = n + nb;
      if (nb == 0.f) return;
      if (n == 0.f) {
        n = nb, m = mb, q = qb;
        return;
      }
      const float d = mb - m;
      m = m + d * (nb / nn);
      q = q + qb + d * d * (n * nb / nn);
      n = nn;
    };
    float vf[TM];  // 1 for this lane's valid pixels, 0 past the end of M
    float nl = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      vf[i] = m0 + wm * WM + 16 * i + fr < g.M ? 1.f : 0.f;
      nl += vf[i];
    }
    // DPP row sums (totals in the row's lane fr = 15, which writes) and a DPP broadcast of the row's
    // first value: no ds_bpermute round trips (see the tiled conv's tile_stats); all TN * 4 chains
    // before one guarded write (a write per j split them into serial groups)
    nl = row_sum15(nl);  // the group's count
    const float inv_n = nl > 0.f ? 1.f / nl : 0.f;
    float cm[TN][4], cq[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) v[i] = (float)(T)acc[j][i][e];
        const float K = row_first(v[0]);
        float sa = 0.f, sq = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float d = (v[i] - K) * vf[i];
          sa += d;
          sq = fmaf(d, d, sq);
        }
        sa = row_sum15(sa);
        sq = row_sum15(sq);
        const float sn = sa * inv_n;
        cm[j][e] = K + sn;
        cq[j][e] = fmaxf(sq - sa * sn, 0.f);
      }
    }
    if (fr == 15) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = wn * WN + 16 * j + 4 * fq + e;
          red[(wm * BN + col) * 3] = nl;
          red[(wm * BN + col) * 3 + 1] = nl > 0.f ? cm[j][e] : 0.f;
          red[(wm * BN + col) * 3 + 2] = nl > 0.f ? cq[j][e] : 0.f;
        }
    }
    __syncthreads();
    for (int t = tid; t < BN; t += NT) {
      float n = 0.f, m = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES_M; ++w)
        chan(n, m, q, red[(w * BN + t) * 3], red[(w * BN + t) * 3 + 1], red[(w * BN + t) * 3 + 2]);
      const int nc = n0 + t;
      if (nc < a.Nout) {
        a.stats[((size_t)tile_m * 2) * a.Nout + nc] = m;
        a.stats[((size_t)tile_m * 2 + 1) * a.Nout + nc] = q;
      }
      if (t == 0 && n0 == 0) a.stats[(size_t)a.ntm * 2 * a.Nout + tile_m] = n;
    }
  }
  clock_end(mc.tp);
}

// ============================================================================ TN (wgrad)
// LDS tiles [BK pixels][cols]; 32-byte windows XOR-swizzled by row so that the transposing
// reads (8 rows x 32 B per half-wave) spread over distinct banks.

// LDS-DMA ring like the NT kernel: one wave-instruction fills 1 KiB = 1024/ROWB pixel rows; lane
// l lands in physical 16-B chunk l % (ROWB/16) of its row and loads the logical chunk given by the
// inverse 32-B-window swizzle, so the transposing fragment reads below stay conflict-light.
template <typename T, int BM, int BN, int WAVES_M, int WAVES_N, int STAGES>
__global__ void __launch_bounds__(256) conv_tn_kernel(TNArgs a) {
  using C = Cfg<T>;
  constexpr int BK = 128 / C::ES;  // pixels per k tile (64 bf16 / 32 f32)
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int QROWB = BM * C::ES, PROWB = BN * C::ES;  // bytes per LDS row
  constexpr int QNW = QROWB / 32, PNW = PROWB / 32;      // 32-B windows per row
  constexpr int QCPR = QROWB / 16, PCPR = PROWB / 16;    // 16-B chunks per row
  constexpr int QRPI = 1024 / QROWB, PRPI = 1024 / PROWB;  // rows per wave-instruction
  constexpr int QI = BK / QRPI / 4, PI = BK / PRPI / 4;    // instructions per wave per tile
  constexpr int PER_TILE = QI + PI;
  static_assert(QI >= 1 && PI >= 1, "tile too small for 4 waves");
  constexpr int TILE_Q = BK * QROWB, TILE_P = BK * PROWB, STAGE = TILE_Q + TILE_P;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];
  clock_begin(a.tp);

  const Gather& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  // 1-D grid over (split, tile), tile fastest.  (Grouping a split's tiles on one XCD cuts the
  // layer-1 HBM fetch 4.6x but ran 1.3x slower: the kernel is issue-bound, not HBM-bound, and
  // the grouped blocks contend for the same L2 lines.)
  const int ntiles = a.ntm * a.ntn;
  const int split = blockIdx.x / ntiles, tile = blockIdx.x - split * ntiles;
  const int tile_m = tile / a.ntn, tile_n = tile % a.ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;  // m: kout, n: (tap, c)
  const int p_begin = split * a.kchunk;
  const int p_end = min(p_begin + a.kchunk, g.M);

  // Buffer-descriptor LDS-DMA loads (out-of-range voffset -> zeros).  Per (lane, instruction) the
  // 16-B column chunk — hence the tap (r,s) and channel of the X gather — is fixed for the whole
  // kernel; per tile only the pixel moves.  With rect_wt, a BK-pixel tile is a rect_wt-wide
  // rectangle of one image, so a lane's pixel is the tile origin (scalar) + a per-lane constant.
  constexpr uint32_t kOOB = 0x80000000u;
  const int qr = lane / QCPR, qc = lane % QCPR;
  const int pr = lane / PCPR, pc = lane % PCPR;
  uint32_t q_col[QI];
  int q_row[QI];
#pragma unroll
  for (int i = 0; i < QI; ++i) {
    const int row = (i * 4 + wave) * QRPI + qr;
    const int lch = 2 * tn_swz<QNW>(row, qc >> 1) + (qc & 1);
    const int col = m0 + lch * C::VEC;
    q_row[i] = row;
    q_col[i] = col < a.Kout ? (uint32_t)(col * C::ES) : kOOB;
  }
  int p_row[PI], p_dh[PI], p_dw[PI], p_coff[PI], p_rr[PI], p_cc[PI];
#pragma unroll
  for (int i = 0; i < PI; ++i) {
    const int row = (i * 4 + wave) * PRPI + pr;
    const int lch = 2 * tn_swz<PNW>(row, pc >> 1) + (pc & 1);
    const int col = n0 + lch * C::VEC;
    const int tap = col >> g.log2Ci, c = col & (g.Ci - 1);
    const int tr = (int)fdiv((uint32_t)tap, g.fd_s);
    p_row[i] = row;
    p_dh[i] = col < a.Ng ? g.off_h + tr * g.ks : -(1 << 28);  // invalid column fails the bounds test
    p_dw[i] = g.off_w + (tap - tr * g.S) * g.ks;
    p_coff[i] = c * C::ES;
    p_rr[i] = a.rect_wt > 0 ? row / a.rect_wt : 0;
    p_cc[i] = a.rect_wt > 0 ? row - p_rr[i] * a.rect_wt : 0;
  }
  const __amdgpu_buffer_rsrc_t qsrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, 0, (uint32_t)((size_t)g.M * a.Kout * C::ES), 0x00020000);
  const __amdgpu_buffer_rsrc_t psrd = __builtin_amdgcn_make_buffer_rsrc((void*)g.base, 0, g.bytes, 0x00020000);
  const int pixstride = g.Ci * C::ES;

  auto issue = [&](int kt, int stage) {
    char* q = smem + stage * STAGE;
    char* p = q + TILE_Q;
    const int pix0 = p_begin + kt * BK;
#pragma unroll
    for (int i = 0; i < QI; ++i) {
      const int px = pix0 + q_row[i];
      const uint32_t voff = px < p_end ? (uint32_t)(px * a.Kout * C::ES) + q_col[i] : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qsrd, (__attribute__((address_space(3))) void*)(q + (i * 4 + wave) * QRPI * QROWB),
                                               16, voff, 0, 0, 0);
    }
    int n0i = 0, oh0 = 0, ow0 = 0;
    if (a.rect_wt > 0) {  // tile origin: wave-uniform
      n0i = (int)fdiv((uint32_t)pix0, g.fd_hw);
      const int rem = pix0 - n0i * g.Ho * g.Wo;
      oh0 = (int)fdiv((uint32_t)rem, g.fd_w);
      ow0 = rem - oh0 * g.Wo;
    }
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const int px = pix0 + p_row[i];
      int n, oh, ow;
      if (a.rect_wt > 0) {
        n = n0i;
        oh = oh0 + p_rr[i];
        ow = ow0 + p_cc[i];
      } else {
        n = (int)fdiv((uint32_t)px, g.fd_hw);
        const int rem = px - n * g.Ho * g.Wo;
        oh = (int)fdiv((uint32_t)rem, g.fd_w);
        ow = rem - oh * g.Wo;
      }
      const int h = oh * g.ms + p_dh[i], w = ow * g.ms + p_dw[i];
      const bool ok = px < p_end && (unsigned)h < (unsigned)g.Hi && (unsigned)w < (unsigned)g.Wi;
      const uint32_t voff = ok ? (uint32_t)(((n * g.Hi + h) * g.Wi + w) * pixstride + p_coff[i]) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(psrd, (__attribute__((address_space(3))) void*)(p + (i * 4 + wave) * PRPI * PROWB),
                                               16, voff, 0, 0, 0);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (p_end - p_begin + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nkt) issue(s, s);
  if (nkt >= STAGES - 1) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_TILE * (STAGES - 2)) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt % STAGES;
    const bool more = kt + STAGES - 1 < nkt;
    if (more) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const char* q = smem + cur * STAGE;
    const char* p = q + TILE_Q;
#pragma unroll
    for (int sub = 0; sub < BK / C::KSUB; ++sub) {
      if constexpr (C::ES == 2) {
        V8<T> pf[TN], qf[TM];
        s16x4 plo[TN], phi[TN], qlo[TM], qhi[TM];
        // lane (fq, fr): rows k = 32 sub + 8 fq + (fr>>2) (+4), cols c0 + 4 (fr&3)
        const int krow = 32 * sub + 8 * fq + (fr >> 2);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int cb = (wn * WN + 16 * j + 4 * (fr & 3)) * 2;
          const int r0 = krow, r1 = krow + 4;
          plo[j] = ds_read_tr16(lds_addr(p + r0 * PROWB + tn_swz<PNW>(r0, cb >> 5) * 32 + (cb & 31)));
          phi[j] = ds_read_tr16(lds_addr(p + r1 * PROWB + tn_swz<PNW>(r1, cb >> 5) * 32 + (cb & 31)));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int cb = (wm * WM + 16 * i + 4 * (fr & 3)) * 2;
          const int r0 = krow, r1 = krow + 4;
          qlo[i] = ds_read_tr16(lds_addr(q + r0 * QROWB + tn_swz<QNW>(r0, cb >> 5) * 32 + (cb & 31)));
          qhi[i] = ds_read_tr16(lds_addr(q + r1 * QROWB + tn_swz<QNW>(r1, cb >> 5) * 32 + (cb & 31)));
        }
        tr_wait();
        typedef short s16x8 __attribute__((ext_vector_type(8)));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const s16x8 v = {plo[j][0], plo[j][1], plo[j][2], plo[j][3], phi[j][0], phi[j][1], phi[j][2], phi[j][3]};
          pf[j] = __builtin_bit_cast(V8<T>, v);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const s16x8 v = {qlo[i][0], qlo[i][1], qlo[i][2], qlo[i][3], qhi[i][0], qhi[i][1], qhi[i][2], qhi[i][3]};
          qf[i] = __builtin_bit_cast(V8<T>, v);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
      } else {
        float pf[TN], qf[TM];
        const int krow = 4 * sub + fq;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int cb = (wn * WN + 16 * j + fr) * 4;
          pf[j] = *(const float*)(p + krow * PROWB + tn_swz<PNW>(krow, cb >> 5) * 32 + (cb & 31));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int cb = (wm * WM + 16 * i + fr) * 4;
          qf[i] = *(const float*)(q + krow * QROWB + tn_swz<QNW>(krow, cb >> 5) * 32 + (cb & 31));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
      }
    }
    if (more) {
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_TILE * (STAGES - 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: slab[split][kout = m][n..n+3]
  float* __restrict__ slab = a.slab + (size_t)split * a.Kout * a.Ng;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + 16 * j + 4 * fq;
    if (n >= a.Ng) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WM + 16 * i + fr;
      if (m < a.Kout) *(f32x4*)(slab + (size_t)m * a.Ng + n) = acc[j][i];
    }
  }
  clock_end(a.tp);
}

// dw_kcrs[k][c][r][s] = sum_z slab[z][k][(r*S+s)*Ci + c]   (c < C real channels)
// im2col mode: column index = (r*S+s)*C + c directly (Ci = padded K of the col matrix).
// Block = QB column-quads x ZL split-lanes (QB * ZL = 256; ZL = the largest power of two <=
// min(16, splits), so no lane idles when there are few splits): lane z0 sums splits z0, z0+ZL, ...
// with 8 independent 16-B loads in flight (the pass is HBM/MALL-bound and needs the bytes in
// flight), then the ZL partial sums are added in a fixed order through LDS -> deterministic.
// The permuted writes to torch's KCRS layout are 4-B scatters (the output is small).
// Workgroups past the reduction's own (blockIdx.x >= nred) do BatchNorm work instead, riding along
// this launch instead of taking launches of their own: fin.C waves (4 per workgroup) finalize the backward of
// the BatchNorm whose sums this conv's backward-data epilogue produced (one channel each), then
// rj.nblk workgroups reduce the backward sums of the BatchNorm whose output gradient this conv's
// backward-data just wrote (the previous block's bn2 / bn2 + downsample-bn).
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int zl_log2,
                                                           int K, int Ng, int C, int R, int S, int Ci, int im2col,
                                                           float* __restrict__ dw, int nred, bn::BnFinDev fin,
                                                           bn::BnRedDev rj) {
  extern __shared__ double ride_lds[];
  if ((int)blockIdx.x >= nred) {
    const int b = blockIdx.x - nred;
    const int nfin = bn::fin_blocks(fin.C);  // one wave per channel
    if (b < nfin) {
      const int c = b * 4 + (int)(threadIdx.x >> 6);
      if (c < fin.C)
        bn::bn_bwd_finalize_w<float>(fin.part, fin.nblk, fin.M, fin.C, c, fin.gamma, fin.mean, fin.invstd, fin.dgamma,
                                     fin.dbeta, fin.coef);
    } else {
      bn::bn_reduce_ride(rj, b - nfin, ride_lds);
    }
    return;
  }
  __shared__ f32x4 part[256];
  const int ZL = 1 << zl_log2, QB = 256 >> zl_log2;
  const int nq = Ng >> 2;
  const int ql = threadIdx.x & (QB - 1), zl = threadIdx.x >> (8 - zl_log2);
  const int qidx = blockIdx.x * QB + ql;  // over K * Ng/4
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const size_t stride = (size_t)K * Ng;
  if (qidx < K * nq) {
    const int k = qidx / nq, col0 = (qidx - k * nq) * 4;
    const float* src = slab + (size_t)k * Ng + col0;
    int z = zl;
    for (; z + 7 * ZL < splits; z += 8 * ZL) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(src + (size_t)(z + u * ZL) * stride);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; z < splits; z += ZL) acc += *(const f32x4*)(src + (size_t)z * stride);
  }
  part[threadIdx.x] = acc;  // [zl][ql]
  __syncthreads();
  if (zl != 0 || qidx >= K * nq) return;
  for (int z = 1; z < ZL; ++z) acc += part[z * QB + ql];
  const int k = qidx / nq, col0 = (qidx - k * nq) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int col = col0 + e;
    int tap, c;
    if (im2col) {
      if (col >= R * S * C) continue;
      tap = col / C;
      c = col - tap * C;
    } else {
      tap = col / Ci;
      c = col - tap * Ci;
    }
    dw[((size_t)k * C + c) * R * S + tap] = acc[e];
  }
}

// Same sum for the (tap, c) column layout (Ci == C), organised so that the permuted KCRS output
// is written with coalesced stores: a block owns output channel k and 64 input channels c0..c0+63,
// i.e. the contiguous run dw[k][c0..c0+63][0..RS-1].  Thread (lane, tap, quad) sums the splits
// lane, lane+ZL, ... of slab[.][k][tap*C + c0 + 4*quad ..+3] (8 loads in flight); the ZL partials
// are added in a fixed order and the block's 64*RS results leave through an LDS transpose.
// Used when the split count is small and the output large (layers 3-4: 4.7 MB, 4 splits), where
// the 4-B scatters of wgrad_reduce_kernel dominated.
__global__ void __launch_bounds__(256) wgrad_reduce_tc_kernel(const float* __restrict__ slab, int splits,
                                                              int zl_log2, int K, int C, int RS,
                                                              float* __restrict__ dw, int nred, bn::BnFinDev fin,
                                                              bn::BnRedDev rj) {
  extern __shared__ double ride_lds[];
  if ((int)blockIdx.x >= nred) {  // riding BatchNorm work (see wgrad_reduce_kernel)
    const int b = blockIdx.x - nred;
    const int nfin = bn::fin_blocks(fin.C);  // one wave per channel
    if (b < nfin) {
      const int c = b * 4 + (int)(threadIdx.x >> 6);
      if (c < fin.C)
        bn::bn_bwd_finalize_w<float>(fin.part, fin.nblk, fin.M, fin.C, c, fin.gamma, fin.mean, fin.invstd, fin.dgamma,
                                     fin.dbeta, fin.coef);
    } else {
      bn::bn_reduce_ride(rj, b - nfin, ride_lds);
    }
    return;
  }
  __shared__ f32x4 part[256];
  __shared__ float outb[64 * 16];
  const int ZL = 1 << zl_log2;
  const int nq = RS * 16;  // (tap, quad) pairs of the block
  const int cgroups = C >> 6;
  const int k = blockIdx.x / cgroups, c0 = (blockIdx.x - k * cgroups) * 64;
  const int t = threadIdx.x;
  const int zl = t / nq, pq = t - zl * nq;  // lanes beyond ZL * nq idle
  const int tap = pq >> 4, q = pq & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const size_t stride = (size_t)K * RS * C;
  if (zl < ZL) {
    const float* src = slab + ((size_t)k * RS + tap) * C + c0 + 4 * q;
    int z = zl;
    for (; z + 7 * ZL < splits; z += 8 * ZL) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(src + (size_t)(z + u * ZL) * stride);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; z < splits; z += ZL) acc += *(const f32x4*)(src + (size_t)z * stride);
    part[t] = acc;
  }
  __syncthreads();
  if (t < nq) {
    for (int z = 1; z < ZL; ++z) acc += part[z * nq + t];
#pragma unroll
    for (int e = 0; e < 4; ++e) outb[(4 * q + e) * RS + tap] = acc[e];
  }
  __syncthreads();
  float* __restrict__ dst = dw + ((size_t)k * C + c0) * RS;
  for (int i = t; i < 64 * RS; i += 256) dst[i] = outb[i];
}

// dw[i] = sum_z slab[z][i] for the slabs that are already in the gradient's KCRS order (the direct
// weight-gradient kernel's; a 1x1 conv's TN slab [K][C] is too): a pure elementwise sum, read and
// written in 16-B pieces with no transpose.  Block = QB quads x ZL split-lanes (QB * ZL = 256); lane
// z sums splits z*NL .. z*NL+NL-1 with all NL loads in flight — indices past the last split are
// clamped to it and their terms masked to zero, so no branch sits between the loads — then the ZL
// lane sums are added in lane order through LDS.  The order depends only on the split count:
// bitwise reproducible.  Workgroups past nred carry the riding BatchNorm work (wgrad_reduce_kernel).
template <int NL>
__global__ void __launch_bounds__(256) wgrad_sum_kernel(const float* __restrict__ slab, int splits, int zl_log2,
                                                        long long E4, float* __restrict__ dw, int nred,
                                                        bn::BnFinDev fin, bn::BnRedDev rj) {
  extern __shared__ double ride_lds[];
  if ((int)blockIdx.x >= nred) {
    const int b = blockIdx.x - nred;
    const int nfin = bn::fin_blocks(fin.C);
    if (b < nfin) {
      const int c = b * 4 + (int)(threadIdx.x >> 6);
      if (c < fin.C)
        bn::bn_bwd_finalize_w<float>(fin.part, fin.nblk, fin.M, fin.C, c, fin.gamma, fin.mean, fin.invstd, fin.dgamma,
                                     fin.dbeta, fin.coef);
    } else {
      bn::bn_reduce_ride(rj, b - nfin, ride_lds);
    }
    return;
  }
  __shared__ f32x4 part[256];
  const int QB = 256 >> zl_log2;
  const int ql = threadIdx.x & (QB - 1), zl = threadIdx.x >> (8 - zl_log2);
  const long long q = (long long)blockIdx.x * QB + ql;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (q < E4) {
    const f32x4* __restrict__ src = (const f32x4*)slab + q;
    const int z0 = zl * NL;
    f32x4 v[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u)  // nontemporal: the slabs are read once (tools/sum_bench.hip: -1.1 us)
      v[u] = __builtin_nontemporal_load(src + (size_t)min(z0 + u, splits - 1) * E4);
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const float m = z0 + u < splits ? 1.f : 0.f;
      acc += v[u] * m;
    }
  }
  if (zl_log2 == 0) {
    if (q < E4) ((f32x4*)dw)[q] = acc;
    return;
  }
  part[threadIdx.x] = acc;  // [zl][ql]
  __syncthreads();
  if (zl != 0 || q >= E4) return;
  for (int z = 1; z < (1 << zl_log2); ++z) acc += part[z * QB + ql];
  ((f32x4*)dw)[q] = acc;
}

// ============================================================================ helpers
// im2col for small-C inputs: col[m][kk] = x[n][oh*st-p+r][ow*st-p+s][c], kk=(r*S+s)*C+c, zero pad.
// One thread per 8 consecutive kk of one row -> one 16-B (bf16) / 2x16-B (f32) store.
template <typename T>
__global__ void im2col_kernel(const T* __restrict__ x, int N, int H, int W, int C, int R, int S, int st,
                              int pad, int Ho, int Wo, int Kp, T* __restrict__ col) {
  const int chunks = Kp >> 3;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // < 2^31 (checked on the host)
  const int total = N * Ho * Wo * chunks;
  if (idx >= total) return;
  const int m = idx / chunks, j = idx - m * chunks;
  const int hw = Ho * Wo;
  const int n = m / hw, rem = m - n * hw;
  const int oh = rem / Wo, ow = rem - oh * Wo;
  const T* __restrict__ xn = x + (size_t)n * H * W * C;
  const int RSC = R * S * C;
  int kk = j * 8;
  int tap = kk / C, c = kk - tap * C;
  int r = tap / S, s = tap - r * S;
  T v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    T val = (T)0.f;
    if (kk < RSC) {
      const int h = oh * st - pad + r, w = ow * st - pad + s;
      if (h >= 0 && h < H && w >= 0 && w < W) val = xn[(h * W + w) * C + c];
    }
    v[e] = val;
    ++kk;
    if (++c == C) {
      c = 0;
      if (++s == S) {
        s = 0;
        ++r;
      }
    }
  }
  T* dst = col + (size_t)m * Kp + j * 8;
  if constexpr (sizeof(T) == 2) {
    *(u32x4*)dst = __builtin_bit_cast(u32x4, v);
  } else {
    *(u32x4*)dst = *(u32x4*)&v[0];
    *(u32x4*)(dst + 4) = *(u32x4*)&v[4];
  }
}

// w_kcrs f32 -> w_krsc (T) [K][R][S][C] (or [K][Kp] im2col layout), w_crsk (T) [C][R][S][K]
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, int K, int C, int R, int S, int st, int pad,
                                   int im2col, int Kp, T* __restrict__ krsc, T* __restrict__ crsk) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int rowlen = im2col ? Kp : R * S * C;
  if (krsc && idx < K * rowlen) {
    const int k = idx / rowlen, j = idx % rowlen;
    float v = 0.f;
    if (j < R * S * C) {
      const int c = j % C, tap = j / C;
      v = w[((size_t)k * C + c) * R * S + tap];
    }
    krsc[idx] = (T)v;
  }
  if (crsk && idx < C * R * S * K) {
    // [C][R][S][K] for stride 1; for stride st the st*st parity classes (ph,pw) back to back, each
    // [C][Rc][Sc][K] with taps r = r0 + st*t, r0 = (ph + pad) % st (see sqr_conv2d_bwd_data)
    int rem = idx, ph = 0, pw = 0, r0 = 0, s0 = 0, Rc = R, Sc = S;
    for (ph = 0; ph < st; ++ph) {
      for (pw = 0; pw < st; ++pw) {
        r0 = (ph + pad) % st;
        s0 = (pw + pad) % st;
        Rc = r0 < R ? (R - r0 + st - 1) / st : 0;
        Sc = s0 < S ? (S - s0 + st - 1) / st : 0;
        const int sz = C * Rc * Sc * K;
        if (rem < sz) goto found;
        rem -= sz;
      }
    }
    return;
  found:
    const int k = rem % K;
    const int u = (rem / K) % Sc;
    const int t = (rem / (K * Sc)) % Rc;
    const int c = rem / (K * Sc * Rc);
    crsk[idx] = (T)w[((size_t)k * C + c) * R * S + (r0 + st * t) * S + (s0 + st * u)];
  }
}

struct PackJob {
  const float* w;
  void* krsc;
  void* crsk;
  int K, C, R, S, st, pad, im2col, Kp, dtype, total;  // total = K*C*R*S source elements
  FastDiv fd_s, fd_r, fd_c;
  int cls_off[4], cls_rc[4], cls_sc[4], cls_r0[4], cls_s0[4];  // dgrad parity classes (st <= 2)
};
struct PackJobs {  // by value as the kernel argument: 20 * 180 B < the 4 KiB argument limit
  PackJob j[20];
};

// pack kernels: one block per (output row, job).  The job's source rows are staged in LDS with
// coalesced fp32 reads and written back in destination order with coalesced stores.
// krsc: block = output channel k: w[k][c][tap] (C*RS floats) -> krsc[k][tap][c] (or im2col [k][Kp]).
template <typename T>
__device__ void pack_krsc_row(const PackJob& jb, int k, float* lds) {
  const int RS = jb.R * jb.S, CRS = jb.C * RS;
  const float* __restrict__ src = jb.w + (size_t)k * CRS;
  for (int i = threadIdx.x; i < CRS; i += 256) lds[i] = src[i];
  __syncthreads();
  const int rowlen = jb.im2col ? jb.Kp : CRS;
  T* __restrict__ dst = (T*)jb.krsc + (size_t)k * rowlen;
  for (int j = threadIdx.x; j < rowlen; j += 256) {
    float v = 0.f;
    if (j < CRS) {
      const int tap = j / jb.C, c = j - tap * jb.C;
      v = lds[c * RS + tap];
    }
    dst[j] = (T)v;
  }
}
// crsk: block = input channel c: gathers w[k][c][tap] for all (k, tap) and writes, per parity
// class, crsk[cls][c][t][u][k] (k innermost -> coalesced)
template <typename T>
__device__ void pack_crsk_row(const PackJob& jb, int c, float* lds) {
  const int RS = jb.R * jb.S, K = jb.K;
  for (int i = threadIdx.x; i < K * RS; i += 256) {
    const int k = i / RS, tap = i - k * RS;
    lds[tap * K + k] = jb.w[((size_t)k * jb.C + c) * RS + tap];
  }
  __syncthreads();
  const int st = jb.st;
  for (int cl = 0; cl < st * st; ++cl) {
    const int Rc = jb.cls_rc[cl], Sc = jb.cls_sc[cl];
    T* __restrict__ dst = (T*)jb.crsk + jb.cls_off[cl] + (size_t)c * Rc * Sc * K;
    for (int i = threadIdx.x; i < Rc * Sc * K; i += 256) {
      const int k = i % K, tu = i / K;
      const int t = tu / Sc, u = tu - t * Sc;
      const int tap = (jb.cls_r0[cl] + st * t) * jb.S + (jb.cls_s0[cl] + st * u);
      dst[i] = (T)lds[tap * K + k];
    }
  }
}

// grid (max(K, C), jobs, 2): z = 0 -> krsc rows, z = 1 -> crsk rows.  LDS: max(C*RS, K*RS) floats.
__global__ void __launch_bounds__(256) pack_weights_batched_kernel(PackJobs jobs) {
  extern __shared__ float plds[];
  const PackJob& jb = jobs.j[blockIdx.y];
  const int row = blockIdx.x;
  if (blockIdx.z == 0) {
    if (!jb.krsc || row >= jb.K) return;
    if (jb.dtype == SQR_DTYPE_BF16) pack_krsc_row<bf16>(jb, row, plds);
    else if (jb.dtype == SQR_DTYPE_F16) pack_krsc_row<f16>(jb, row, plds);
    else pack_krsc_row<float>(jb, row, plds);
  } else {
    if (!jb.crsk || row >= jb.C) return;
    if (jb.dtype == SQR_DTYPE_BF16) pack_crsk_row<bf16>(jb, row, plds);
    else if (jb.dtype == SQR_DTYPE_F16) pack_crsk_row<f16>(jb, row, plds);
    else pack_crsk_row<float>(jb, row, plds);
  }
}

}  // namespace conv
}  // namespace sqr

using namespace sqr;
using namespace sqr::conv;

// ============================================================================ host planning
namespace {

struct Shape {
  int Ho, Wo, M;
  bool im2col;  // input channels < 8 -> explicit im2col + 1x1
  int Kp;       // im2col K (R*S*C rounded up to a power of two >= 64)
  int ES;
};

bool is_pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }
int ilog2(int x) {
  int l = 0;
  while ((1 << l) < x) ++l;
  return l;
}

int check_desc(const sqr_conv_desc* d, Shape* sh) {
  SQR_CHECK_ARG(d, "conv2d: null descriptor");
  SQR_CHECK_ARG(d->N >= 1 && d->C >= 1 && d->H >= 1 && d->W >= 1 && d->K >= 1 && d->R >= 1 && d->S >= 1,
                "conv2d: non-positive dims");
  SQR_CHECK_ARG(d->stride >= 1 && d->pad >= 0, "conv2d: bad stride/pad");
  SQR_CHECK_ARG(d->dtype == SQR_DTYPE_F32 || d->dtype == SQR_DTYPE_BF16 || d->dtype == SQR_DTYPE_F16,
                "conv2d: bad dtype %d", d->dtype);
  sh->ES = d->dtype == SQR_DTYPE_F32 ? 4 : 2;
  sh->Ho = (d->H + 2 * d->pad - d->R) / d->stride + 1;
  sh->Wo = (d->W + 2 * d->pad - d->S) / d->stride + 1;
  SQR_CHECK_ARG(sh->Ho >= 1 && sh->Wo >= 1, "conv2d: empty output");
  const long long M = (long long)d->N * sh->Ho * sh->Wo;
  const long long Min = (long long)d->N * d->H * d->W;
  SQR_CHECK_ARG(M < (1ll << 31) && Min < (1ll << 31), "conv2d: too many pixels");
  SQR_CHECK_ARG(d->C >= 8 || M * 64 < (1ll << 31), "conv2d: too many pixels for the im2col path");
  sh->M = (int)M;
  sh->im2col = d->C < 8;
  sh->Kp = 64;  // im2col K: next power of two >= max(64, R*S*C) (the gather needs a power-of-2 row)
  while (sh->Kp < d->R * d->S * d->C) sh->Kp *= 2;
  // 32-bit buffer offsets: every operand tensor (and the im2col matrix) must stay below 2 GiB
  const long long es = d->dtype == SQR_DTYPE_F32 ? 4 : 2;
  SQR_CHECK_ARG(Min * d->C * es < (1ll << 31) && M * d->K * es < (1ll << 31) &&
                    (!sh->im2col || M * sh->Kp * es < (1ll << 31)),
                "conv2d: tensors larger than 2 GiB are not supported");
  const int vec = 16 / sh->ES;
  SQR_CHECK_ARG(sh->im2col || (is_pow2(d->C) && d->C % vec == 0), "conv2d: C=%d must be a power of 2 >= 8", d->C);
  SQR_CHECK_ARG(d->K % 8 == 0 && is_pow2(d->K), "conv2d: K=%d must be a power of 2 >= 8", d->K);
  SQR_CHECK_ARG(d->R * d->S <= 64, "conv2d: at most 64 taps");
  return 0;
}

Gather make_gather(const void* base, int Hi, int Wi, int Ci, int Ho, int Wo, int ms, int off_h, int off_w, int ks,
                   int R, int S, int N, int es) {
  Gather g;
  g.base = base;
  g.Hi = Hi;
  g.Wi = Wi;
  g.Ci = Ci;
  g.log2Ci = ilog2(Ci);
  g.Ho = Ho;
  g.Wo = Wo;
  g.ms = ms;
  g.off_h = off_h;
  g.off_w = off_w;
  g.ks = ks;
  g.R = R;
  g.S = S;
  g.M = N * Ho * Wo;
  g.fd_hw = make_fastdiv((uint32_t)(Ho * Wo));
  g.fd_w = make_fastdiv((uint32_t)Wo);
  g.fd_s = make_fastdiv((uint32_t)S);
  g.bytes = (uint32_t)((size_t)N * Hi * Wi * Ci * es);
  return g;
}

int nt_cfg(int M, int N, bool bf16) {
  auto nblk = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (N >= 128 && nblk(128, 128) >= 512) return 0;
  // one 128x128 tile per CU: 8 waves + a 4-deep ring (ResNetSQ layer3 convs, layer4's strided
  // dgrad: 8-13 % faster than 128x64 / 4 waves, measured scratch/nt_tune.py)
  if (bf16 && N >= 128 && nblk(128, 128) >= 256) return 5;
  if (nblk(128, 64) >= 512) return 1;
  if (N >= 128 && nblk(64, 128) >= 512) return 2;
  return 3;
}

// tile configs of launch_nt: BM, BN, threads
const int kNtBM[8] = {128, 128, 64, 64, 256, 128, 128, 128};
const int kNtBN[8] = {128, 64, 128, 64, 128, 128, 128, 64};
const int kNtThreads[8] = {256, 256, 256, 256, 512, 512, 256, 512};

int nt_pick(int M, int N, bool bf16) {
  const int cfg = nt_cfg(M, N, bf16);
  return cfg < 0 || cfg > 7 ? 0 : cfg;
}

// one launch for ncls NT GEMMs of the same output width (tile config from their total M)
template <typename T>
int launch_nt(NTArgs* cl, int ncls, hipStream_t st) {
  // tile choice: biggest tile that still gives >= 2 workgroups per CU (512), one 8-wave 128x128 tile
  // per CU, else the smallest
  int M = 0;
  for (int i = 0; i < ncls; ++i) M += cl[i].g.M;
  const int N = cl[0].Nout;
  const int cfg = nt_pick(M, N, sizeof(T) == 2);
  const int bm = kNtBM[cfg], bn = kNtBN[cfg];
  NTMulti mc;
  int total = 0;
  for (int i = 0; i < ncls; ++i) {
    cl[i].ntm = (cl[i].g.M + bm - 1) / bm;
    cl[i].ntn = (N + bn - 1) / bn;
    mc.c[i] = cl[i];
    mc.start[i] = total;
    total += cl[i].ntm * cl[i].ntn;
  }
  for (int i = ncls; i < 4; ++i) mc.start[i] = total;
  mc.ncls = ncls;
  mc.tp = probe_clock_take();
  const dim3 grid(total), blk(kNtThreads[cfg]);
  probe_begin(st);
  switch (cfg) {
    case 0: hipLaunchKernelGGL((conv_nt_kernel<T, 128, 128, 2, 2, 2>), grid, blk, 0, st, mc); break;
    case 1: hipLaunchKernelGGL((conv_nt_kernel<T, 128, 64, 4, 1, 3>), grid, blk, 0, st, mc); break;
    case 2: hipLaunchKernelGGL((conv_nt_kernel<T, 64, 128, 1, 4, 3>), grid, blk, 0, st, mc); break;
    case 3: hipLaunchKernelGGL((conv_nt_kernel<T, 64, 64, 2, 2, 3>), grid, blk, 0, st, mc); break;
    case 4: hipLaunchKernelGGL((conv_nt_kernel<T, 256, 128, 4, 2, 3>), grid, blk, 0, st, mc); break;
    case 5: hipLaunchKernelGGL((conv_nt_kernel<T, 128, 128, 2, 4, 4>), grid, blk, 0, st, mc); break;
    case 6: hipLaunchKernelGGL((conv_nt_kernel<T, 128, 128, 2, 2, 4>), grid, blk, 0, st, mc); break;
    default: hipLaunchKernelGGL((conv_nt_kernel<T, 128, 64, 4, 2, 5>), grid, blk, 0, st, mc); break;
  }
  probe_end(st);
  SQR_HIP_LAUNCH_CHECK("conv_nt_kernel");
  return 0;
}

struct TNPlan {
  int bm, bn, ntm, ntn, splits, kchunk;
};

TNPlan plan_tn(int Kout, int Ng, int Mpix, int ES) {
  TNPlan p;
  p.bm = Kout >= 128 ? 128 : 64;
  p.bn = Ng >= 128 ? 128 : 64;
  p.ntm = (Kout + p.bm - 1) / p.bm;
  p.ntn = (Ng + p.bn - 1) / p.bn;
  const int BK = 128 / ES;
  const int tiles = p.ntm * p.ntn;
  int splits = (512 + tiles - 1) / tiles;  // ~2 workgroups per CU
  const int maxs = (Mpix + BK - 1) / BK;
  splits = splits < 1 ? 1 : (splits > maxs ? maxs : splits);
  int kchunk = (Mpix + splits - 1) / splits;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  p.splits = (Mpix + kchunk - 1) / kchunk;
  p.kchunk = kchunk;
  return p;
}

template <typename T>
int launch_tn(TNArgs a, const TNPlan& p, hipStream_t st) {
  a.ntm = p.ntm;
  a.ntn = p.ntn;
  a.kchunk = p.kchunk;
  a.tp = probe_clock_take();
  const dim3 grid(p.ntm * p.ntn * p.splits), blk(256);
  probe_begin(st);
  if (p.bm == 128 && p.bn == 128) hipLaunchKernelGGL((conv_tn_kernel<T, 128, 128, 2, 2, 2>), grid, blk, 0, st, a);
  else if (p.bm == 128) hipLaunchKernelGGL((conv_tn_kernel<T, 128, 64, 4, 1, 3>), grid, blk, 0, st, a);
  else if (p.bn == 128) hipLaunchKernelGGL((conv_tn_kernel<T, 64, 128, 1, 4, 3>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((conv_tn_kernel<T, 64, 64, 2, 2, 3>), grid, blk, 0, st, a);
  probe_end(st);
  SQR_HIP_LAUNCH_CHECK("conv_tn_kernel");
  return 0;
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// split-lanes: the largest power of two <= min(cap, splits)
int reduce_zl_log2(int splits, int cap = 16) {
  int l = 0;
  while ((2 << l) <= cap && (2 << l) <= splits) ++l;
  return l;
}

// fixed-order sum of KCRS-ordered slabs (E floats each, E % 4 == 0): NL = loads per lane (the
// next power of two >= splits, at most 16), ZL = lanes per quad (the next power of two >=
// splits / 16)
int launch_wgrad_sum(const float* slab, int splits, long long E, float* dw, hipStream_t st,
                     const bn::BnFinDev* fin = nullptr, const bn::BnRedDev* red = nullptr, size_t red_lds = 0) {
  bn::BnFinDev f = {};
  bn::BnRedDev r = {};
  if (fin) f = *fin;
  if (red) r = *red;
  const int nride = (fin ? bn::fin_blocks(fin->C) : 0) + (red ? red->nblk : 0);
  const size_t lds = red ? red_lds : 0;
  int nl = 1;
  while (nl < splits && nl < 16) nl *= 2;
  int zlg = 0;
  while ((16 << zlg) < splits && zlg < 8) ++zlg;
  SQR_CHECK_ARG(splits <= (16 << zlg), "wgrad_sum: %d splits", splits);
  const long long E4 = E / 4;
  const int QB = 256 >> zlg;
  const int nred = (int)((E4 + QB - 1) / QB);
  const dim3 grid(nred + nride), blk(256);
  switch (nl) {
    case 1: hipLaunchKernelGGL(wgrad_sum_kernel<1>, grid, blk, lds, st, slab, splits, zlg, E4, dw, nred, f, r); break;
    case 2: hipLaunchKernelGGL(wgrad_sum_kernel<2>, grid, blk, lds, st, slab, splits, zlg, E4, dw, nred, f, r); break;
    case 4: hipLaunchKernelGGL(wgrad_sum_kernel<4>, grid, blk, lds, st, slab, splits, zlg, E4, dw, nred, f, r); break;
    case 8: hipLaunchKernelGGL(wgrad_sum_kernel<8>, grid, blk, lds, st, slab, splits, zlg, E4, dw, nred, f, r); break;
    default: hipLaunchKernelGGL(wgrad_sum_kernel<16>, grid, blk, lds, st, slab, splits, zlg, E4, dw, nred, f, r); break;
  }
  SQR_HIP_LAUNCH_CHECK("wgrad_sum_kernel");
  return 0;
}

// fixed-order split-K sum of the weight-gradient slabs into torch's [K][C][R][S]
int launch_wgrad_reduce(const float* slab, int splits, int K, int Ng, int C, int R, int S, int Ci, int im2col,
                        float* dw, hipStream_t st, const bn::BnFinDev* fin = nullptr,
                        const bn::BnRedDev* red = nullptr, size_t red_lds = 0) {
  const int RS = R * S;
  bn::BnFinDev f = {};
  bn::BnRedDev r = {};
  if (fin) f = *fin;
  if (red) r = *red;
  const int nride = (fin ? bn::fin_blocks(fin->C) : 0) + (red ? red->nblk : 0);
  const size_t lds = red ? red_lds : 0;
  if (!im2col && Ci == C && C % 64 == 0 && RS <= 16 && splits <= 16) {
    const int zlg = reduce_zl_log2(splits, 256 / (RS * 16));
    const int nred = K * (C / 64);
    hipLaunchKernelGGL(wgrad_reduce_tc_kernel, dim3(nred + nride), dim3(256), lds, st, slab, splits, zlg, K, C, RS, dw,
                       nred, f, r);
    SQR_HIP_LAUNCH_CHECK("wgrad_reduce_tc_kernel");
    return 0;
  }
  const int total = K * (Ng / 4);
  const int zlg = reduce_zl_log2(splits);
  const int nred = (total + (256 >> zlg) - 1) / (256 >> zlg);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(nred + nride), dim3(256), lds, st, slab, splits, zlg, K, Ng, C, R, S,
                     Ci, im2col, dw, nred, f, r);
  SQR_HIP_LAUNCH_CHECK("wgrad_reduce_kernel");
  return 0;
}

}  // namespace

// ============================================================================ C ABI
extern "C" int sqr_conv2d_out_hw(const sqr_conv_desc* d, int* Ho, int* Wo) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(Ho && Wo, "conv2d_out_hw: null output");
  *Ho = sh.Ho;
  *Wo = sh.Wo;
  return 0;
}

// 16-bit 3x3 / stride 1 / pad 1 (the direct kernels' domain; they decline other shapes themselves)
static bool direct3(const sqr_conv_desc* d, const Shape& sh) {
  return !sh.im2col && d->dtype != SQR_DTYPE_F32 && d->R == 3 && d->S == 3 && d->stride == 1 && d->pad == 1;
}
// the direct forward kernel's stride-2 mode (the first conv of layers 2-4)
static bool direct3s2(const sqr_conv_desc* d, const Shape& sh) {
  return !sh.im2col && d->dtype != SQR_DTYPE_F32 && d->R == 3 && d->S == 3 && d->stride == 2 && d->pad == 1 &&
         d->H == 2 * sh.Ho && d->W == 2 * sh.Wo;
}
// the direct weight-gradient kernel also takes stride 2 (the first conv of layers 2-4)
static bool direct3w(const sqr_conv_desc* d, const Shape& sh) {
  return !sh.im2col && d->dtype != SQR_DTYPE_F32 && d->R == 3 && d->S == 3 && (d->stride == 1 || d->stride == 2) &&
         d->pad == 1;
}

extern "C" size_t sqr_conv2d_workspace_bytes(const sqr_conv_desc* d, int which) {
  Shape sh;
  if (check_desc(d, &sh)) return 0;
  const size_t col = sh.im2col ? align_up((size_t)sh.M * sh.Kp * sh.ES) : 0;
  if (which == 0) return col;
  if (which == 1) return 0;
  const int Ng = sh.im2col ? sh.Kp : d->R * d->S * d->C;
  const TNPlan p = plan_tn(d->K, Ng, sh.M, sh.ES);
  size_t slab = (size_t)p.splits * d->K * Ng * sizeof(float);
  if (direct3w(d, sh)) {
    const size_t s3 = conv3w_slab_bytes(d->N, d->H, d->W, d->C, d->K, d->stride);
    slab = s3 > slab ? s3 : slab;
  }
  return col + align_up(slab);
}

extern "C" int sqr_conv2d_pack_weight(const float* w_kcrs, const sqr_conv_desc* d, void* w_krsc, void* w_crsk,
                                      void* stream) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(w_kcrs && (w_krsc || w_crsk), "conv2d_pack_weight: null pointer");
  SQR_CHECK_ARG(!(sh.im2col && w_crsk), "conv2d_pack_weight: no dgrad weights for C<8 (im2col) convs");
  const int total = d->K * (sh.im2col ? sh.Kp : d->R * d->S * d->C);
  const int blocks = (total + 255) / 256;
  hipStream_t st = as_stream(stream);
  if (d->dtype != SQR_DTYPE_F32)
    SQR_DISPATCH16(d->dtype, T,
                   hipLaunchKernelGGL((pack_weight_kernel<T>), dim3(blocks), dim3(256), 0, st, w_kcrs, d->K, d->C,
                                      d->R, d->S, d->stride, d->pad, (int)sh.im2col, sh.Kp, (T*)w_krsc, (T*)w_crsk));
  else
    hipLaunchKernelGGL((pack_weight_kernel<float>), dim3(blocks), dim3(256), 0, st, w_kcrs, d->K, d->C, d->R,
                       d->S, d->stride, d->pad, (int)sh.im2col, sh.Kp, (float*)w_krsc, (float*)w_crsk);
  SQR_HIP_LAUNCH_CHECK("pack_weight_kernel");
  return 0;
}

template <typename T>
static int im2col(const void* x, const sqr_conv_desc* d, const Shape& sh, void* col, hipStream_t st) {
  const size_t total = (size_t)sh.M * (sh.Kp / 8);
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL((im2col_kernel<T>), dim3(blocks), dim3(256), 0, st, (const T*)x, d->N, d->H, d->W, d->C,
                     d->R, d->S, d->stride, d->pad, sh.Ho, sh.Wo, sh.Kp, (T*)col);
  SQR_HIP_LAUNCH_CHECK("im2col_kernel");
  return 0;
}

static int conv_fwd_impl(const void* x, const void* w_krsc, void* y, const sqr_conv_desc* d, float* stats,
                         int* stats_rows, void* workspace, size_t workspace_bytes, void* stream) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(x && w_krsc && y, "conv2d_fwd: null pointer");
  hipStream_t st = as_stream(stream);
  NTArgs a;
  a.w = w_krsc;
  a.Nout = d->K;
  a.out = y;
  a.os = 1;
  a.oph = a.opw = 0;
  a.oH = sh.Ho;
  a.oW = sh.Wo;
  if (direct3(d, sh)) {
    rc = conv3_launch(d->dtype, x, w_krsc, y, d->N, d->H, d->W, d->C, d->K, 0, stats, stats_rows, st);
    if (rc != kNotHandled) return rc;  // launched (0) or failed; else the shape is not covered
  }
  if (direct3s2(d, sh)) {
    rc = conv3_launch(d->dtype, x, w_krsc, y, d->N, d->H, d->W, d->C, d->K, 0, stats, stats_rows, st, nullptr,
                      nullptr, 2);
    if (rc != kNotHandled) return rc;
  }
  a.stats = stats;
  if (stats_rows) {  // one partial row per M tile of the config launch_nt will pick
    const int bm = kNtBM[nt_pick(sh.M, d->K, d->dtype != SQR_DTYPE_F32)];
    *stats_rows = (sh.M + bm - 1) / bm;
  }
  if (sh.im2col) {
    const size_t need = sqr_conv2d_workspace_bytes(d, 0);
    if (workspace_bytes < need || !workspace) {
      set_error("conv2d_fwd: workspace %zu < %zu", workspace_bytes, need);
      return SQR_E_WORKSPACE;
    }
    if (d->dtype == SQR_DTYPE_F32) rc = im2col<float>(x, d, sh, workspace, st);
    else SQR_DISPATCH16(d->dtype, T, rc = im2col<T>(x, d, sh, workspace, st));
    if (rc) return rc;
    a.g = make_gather(workspace, sh.Ho, sh.Wo, sh.Kp, sh.Ho, sh.Wo, 1, 0, 0, 1, 1, 1, d->N, sh.ES);
    a.Kg = sh.Kp;
  } else {
    a.g = make_gather(x, d->H, d->W, d->C, sh.Ho, sh.Wo, d->stride, -d->pad, -d->pad, 1, d->R, d->S, d->N, sh.ES);
    a.Kg = d->R * d->S * d->C;
  }
  if (d->dtype == SQR_DTYPE_F32) return launch_nt<float>(&a, 1, st);
  SQR_DISPATCH16(d->dtype, T, rc = launch_nt<T>(&a, 1, st));
  return rc;
}

extern "C" int sqr_conv2d_fwd(const void* x, const void* w_krsc, void* y, const sqr_conv_desc* d,
                              void* workspace, size_t workspace_bytes, void* stream) {
  return conv_fwd_impl(x, w_krsc, y, d, nullptr, nullptr, workspace, workspace_bytes, stream);
}

extern "C" size_t sqr_conv2d_stats_floats(const sqr_conv_desc* d) {
  Shape sh;
  if (check_desc(d, &sh)) return 0;
  return (size_t)((sh.M + 63) / 64) * (2 * d->K + 1);  // rows of (mean, M2) + a count per row
}

extern "C" int sqr_conv2d_fwd_stats(const void* x, const void* w_krsc, void* y, const sqr_conv_desc* d, float* stats,
                                    int* stats_rows, void* workspace, size_t workspace_bytes, void* stream) {
  SQR_CHECK_ARG(stats && stats_rows, "conv2d_fwd_stats: null stats output");
  return conv_fwd_impl(x, w_krsc, y, d, stats, stats_rows, workspace, workspace_bytes, stream);
}

extern "C" int sqr_conv2d_fwd_stats_bnin(const void* x_pre, const float* coef, void* x_act, uint8_t* x_mask,
                                         const void* w_krsc, void* y, const sqr_conv_desc* d, float* stats,
                                         int* stats_rows, void* stream) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(x_pre && coef && w_krsc && y && stats && stats_rows && (!x_act) == (!x_mask),
                "conv2d_fwd_stats_bnin: null pointer (x_act and x_mask: both or neither)");
  if (!direct3(d, sh)) {
    set_error("conv2d_fwd_stats_bnin: only 16-bit 3x3 / stride 1 / pad 1 convs");
    return SQR_E_UNSUPPORTED;
  }
  const BnInArgs b = {coef, x_act, x_mask};
  rc = conv3_launch(d->dtype, x_pre, w_krsc, y, d->N, d->H, d->W, d->C, d->K, 0, stats, stats_rows, as_stream(stream),
                    nullptr, nullptr, 1, nullptr, &b);
  if (rc == kNotHandled) {
    set_error(x_act ? "conv2d_fwd_stats_bnin: side outputs only on the persistent layer-1 kernel's shapes (64 -> 64 "
                      "channels, 64- or 128-wide maps)"
                    : "conv2d_fwd_stats_bnin: no direct kernel with apply-on-load for this shape "
                      "(sqr_conv2d_bnin_nso_supported)");
    return SQR_E_UNSUPPORTED;
  }
  return rc;
}

// dgrad parity class (ph, pw) of a stride-st conv: taps r = r0 + st*t with (ph + pad - r) % st == 0
struct DgradClass {
  int r0, Rc, s0, Sc, Hc, Wc, off_h, off_w;
};
static DgradClass dgrad_class(const sqr_conv_desc* d, int ph, int pw) {
  DgradClass c;
  const int st = d->stride;
  c.r0 = (ph + d->pad) % st;
  c.s0 = (pw + d->pad) % st;
  c.Rc = c.r0 < d->R ? (d->R - c.r0 + st - 1) / st : 0;
  c.Sc = c.s0 < d->S ? (d->S - c.s0 + st - 1) / st : 0;
  c.Hc = ph < d->H ? (d->H - ph + st - 1) / st : 0;
  c.Wc = pw < d->W ? (d->W - pw + st - 1) / st : 0;
  c.off_h = (ph + d->pad - c.r0) / st;
  c.off_w = (pw + d->pad - c.s0) / st;
  return c;
}

static int bwd_data_gemm(const void* dy, const void* w_crsk, void* dx, const sqr_conv_desc* d, const Shape& sh,
                         hipStream_t st);

// dx += addend over n elements (the implicit-GEMM backward-data path of sqr_conv2d_bwd_data_acc;
// the direct kernels add in their epilogues)
template <typename T>
__global__ void __launch_bounds__(256) add_inplace_kernel(T* __restrict__ dx, const T* __restrict__ addend, long long n) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 4 <= n) {
#pragma unroll
    for (int e = 0; e < 4; ++e) dx[i + e] = (T)((float)dx[i + e] + (float)addend[i + e]);
  } else {
    for (long long e = i; e < n; ++e) dx[e] = (T)((float)dx[e] + (float)addend[e]);
  }
}

static int bwd_data_impl(const void* dy, const void* w_crsk, void* dx, const void* addend, const sqr_conv_desc* d,
                         void* stream) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(!sh.im2col, "conv2d_bwd_data: C=%d < 8 not supported", d->C);
  SQR_CHECK_ARG(dy && w_crsk && dx, "conv2d_bwd_data: null pointer");
  SQR_CHECK_ARG(addend != dx, "conv2d_bwd_data_acc: addend must not alias dx");
  hipStream_t st = as_stream(stream);
  if (direct3(d, sh)) {
    rc = conv3_launch(d->dtype, dy, w_crsk, dx, d->N, d->H, d->W, d->K, d->C, 1, nullptr, nullptr, st, addend);
    if (rc != kNotHandled) return rc;
  }
  if (d->dtype != SQR_DTYPE_F32 && d->R == 3 && d->S == 3 && d->stride == 2 && d->pad == 1 &&
      d->H == 2 * sh.Ho && d->W == 2 * sh.Wo) {
    const int off[4] = {0, d->C * d->K, 3 * d->C * d->K, 5 * d->C * d->K};  // classes of 1, 2, 2, 4 taps
    rc = conv3s2_dgrad_launch(d->dtype, dy, w_crsk, off, dx, d->N, sh.Ho, sh.Wo, d->K, d->C, st, addend);
    if (rc != kNotHandled) return rc;
  }
  rc = bwd_data_gemm(dy, w_crsk, dx, d, sh, st);
  if (rc || !addend) return rc;
  const long long n = (long long)d->N * d->H * d->W * d->C;
  const unsigned grid = (unsigned)((n + 1023) / 1024);
  if (d->dtype == SQR_DTYPE_F32)
    hipLaunchKernelGGL(add_inplace_kernel<float>, dim3(grid), dim3(256), 0, st, (float*)dx, (const float*)addend, n);
  else
    SQR_DISPATCH16(d->dtype, T, hipLaunchKernelGGL(add_inplace_kernel<T>, dim3(grid), dim3(256), 0, st, (T*)dx,
                                                   (const T*)addend, n));
  SQR_HIP_LAUNCH_CHECK("add_inplace_kernel");
  return 0;
}

extern "C" int sqr_conv2d_bwd_data(const void* dy, const void* w_crsk, void* dx, const sqr_conv_desc* d,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  return bwd_data_impl(dy, w_crsk, dx, nullptr, d, stream);
}

// dx[n, 2i, 2j, c] += addend_c[n, i, j, c]: the fallback of sqr_conv2d_bwd_data_acc_s2
template <typename T>
__global__ void __launch_bounds__(256) add_s2_compact_kernel(T* __restrict__ dx, const T* __restrict__ ac, int Ho,
                                                             int Wo, int C, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;  // one element of addend_c
  if (i >= n) return;
  const long long pix = i / C;
  const int c = (int)(i - pix * C);
  const long long img = pix / ((long long)Ho * Wo);
  const int rem = (int)(pix - img * Ho * Wo), y = rem / Wo, x = rem - y * Wo;
  const size_t o = ((size_t)(img * 2 * Ho + 2 * y) * (2 * Wo) + 2 * x) * C + c;
  dx[o] = (T)((float)dx[o] + (float)ac[i]);
}

extern "C" int sqr_conv2d_bwd_data_acc_s2(const void* dy, const void* w_crsk, void* dx, const void* addend_c,
                                          const sqr_conv_desc* d, void* workspace, size_t workspace_bytes,
                                          void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(dy && w_crsk && dx && addend_c, "conv2d_bwd_data_acc_s2: null pointer");
  SQR_CHECK_ARG(d->stride == 2 && d->H == 2 * sh.Ho && d->W == 2 * sh.Wo && !sh.im2col,
                "conv2d_bwd_data_acc_s2: needs a stride-2 conv with H = 2 Ho, W = 2 Wo");
  hipStream_t st = as_stream(stream);
  if (d->dtype != SQR_DTYPE_F32 && d->R == 3 && d->S == 3 && d->pad == 1) {
    const int off[4] = {0, d->C * d->K, 3 * d->C * d->K, 5 * d->C * d->K};
    rc = conv3s2_dgrad_launch(d->dtype, dy, w_crsk, off, dx, d->N, sh.Ho, sh.Wo, d->K, d->C, st, addend_c, 1);
    if (rc != kNotHandled) return rc;
  }
  rc = bwd_data_impl(dy, w_crsk, dx, nullptr, d, stream);
  if (rc) return rc;
  const long long n = (long long)d->N * sh.Ho * sh.Wo * d->C;
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (d->dtype == SQR_DTYPE_F32)
    hipLaunchKernelGGL(add_s2_compact_kernel<float>, dim3(grid), dim3(256), 0, st, (float*)dx, (const float*)addend_c,
                       sh.Ho, sh.Wo, d->C, n);
  else
    SQR_DISPATCH16(d->dtype, T, hipLaunchKernelGGL(add_s2_compact_kernel<T>, dim3(grid), dim3(256), 0, st, (T*)dx,
                                                   (const T*)addend_c, sh.Ho, sh.Wo, d->C, n));
  SQR_HIP_LAUNCH_CHECK("add_s2_compact_kernel");
  return 0;
}

extern "C" int sqr_conv2d_bwd_data_acc(const void* dy, const void* w_crsk, void* dx, const void* addend,
                                       const sqr_conv_desc* d, void* workspace, size_t workspace_bytes, void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  SQR_CHECK_ARG(addend, "conv2d_bwd_data_acc: null addend");
  return bwd_data_impl(dy, w_crsk, dx, addend, d, stream);
}

extern "C" int sqr_conv2d_bwd_data_acc_masked(const void* dy, const void* w_crsk, void* dx, const void* addend,
                                              const uint8_t* addend_mask, const sqr_conv_desc* d, void* workspace,
                                              size_t workspace_bytes, void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(dy && w_crsk && dx && addend && addend_mask, "conv2d_bwd_data_acc_masked: null pointer");
  SQR_CHECK_ARG(addend != dx, "conv2d_bwd_data_acc_masked: addend must not alias dx");
  rc = kNotHandled;
  if (!sh.im2col && direct3(d, sh))
    rc = conv3_launch(d->dtype, dy, w_crsk, dx, d->N, d->H, d->W, d->K, d->C, 1, nullptr, nullptr, as_stream(stream),
                      addend, nullptr, 1, addend_mask);
  if (rc == kNotHandled) {
    set_error("conv2d_bwd_data_acc_masked: only the direct 3x3 / stride-1 16-bit kernels take a masked addend");
    return SQR_E_UNSUPPORTED;
  }
  return rc;
}

extern "C" size_t sqr_conv2d_bwd_data_bn_stats_floats(const sqr_conv_desc* d) {
  Shape sh;
  if (check_desc(d, &sh)) return 0;
  const long long M = (long long)d->N * d->H * d->W;
  size_t rows = (size_t)((M + 63) / 64);
  const size_t rf = bn_mask_reduce_rows(M, d->C);
  rows = rows < rf ? rf : rows;
  rows = rows < 1024 ? 1024 : rows;
  return rows * 2 * d->C;
}

extern "C" int sqr_conv2d_bwd_data_bn(const void* dy, const void* w_crsk, void* g_out, const void* bn_x,
                                      const uint8_t* relu_mask, const float* bn_mean, float* stats, int* stats_rows,
                                      const sqr_conv_desc* d, void* workspace, size_t workspace_bytes, void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(!sh.im2col, "conv2d_bwd_data_bn: C=%d < 8 not supported", d->C);
  SQR_CHECK_ARG(dy && w_crsk && g_out && bn_x && relu_mask && bn_mean && stats && stats_rows,
                "conv2d_bwd_data_bn: null pointer");
  hipStream_t st = as_stream(stream);
  if (direct3(d, sh)) {
    const BnbArgs bnb = {bn_x, relu_mask, bn_mean};
    rc = conv3_launch(d->dtype, dy, w_crsk, g_out, d->N, d->H, d->W, d->K, d->C, 1, stats, stats_rows, st, nullptr,
                      &bnb);
    if (rc != kNotHandled) return rc;
  }
  rc = bwd_data_impl(dy, w_crsk, g_out, nullptr, d, stream);
  if (rc) return rc;
  return bn_mask_reduce(g_out, bn_x, relu_mask, bn_mean, (long long)d->N * d->H * d->W, d->C, d->dtype, stats,
                        stats_rows, st);
}

extern "C" int sqr_conv2d_bnin_nso_supported(const sqr_conv_desc* d) {
  Shape sh;
  if (!d || check_desc(d, &sh) || !direct3(d, sh)) return 0;
  return conv3_bnin_nso_ok(d->N, d->H, d->W, d->C, d->K);
}

extern "C" int sqr_conv2d_bwd_data_bn_act(const void* dy, const void* w_crsk, void* g_out, const void* bn_x,
                                          const float* bn_coef, const float* bn_mean, void* act_out, float* stats,
                                          int* stats_rows, const sqr_conv_desc* d, void* stream) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(dy && w_crsk && g_out && bn_x && bn_coef && bn_mean && stats && stats_rows,
                "conv2d_bwd_data_bn_act: null pointer");
  if (!direct3(d, sh)) {
    set_error("conv2d_bwd_data_bn_act: only 16-bit 3x3 / stride 1 / pad 1 convs");
    return SQR_E_UNSUPPORTED;
  }
  BnbArgs bnb = {bn_x, nullptr, bn_mean};
  bnb.coef = bn_coef;
  bnb.act = act_out;
  rc = conv3_launch(d->dtype, dy, w_crsk, g_out, d->N, d->H, d->W, d->K, d->C, 1, stats, stats_rows, as_stream(stream),
                    nullptr, &bnb);
  if (rc == kNotHandled) {
    set_error("conv2d_bwd_data_bn_act: no direct kernel for this shape (sqr_conv2d_bnin_nso_supported)");
    return SQR_E_UNSUPPORTED;
  }
  return rc;
}

// implicit-GEMM backward-data over the output parity classes
static int bwd_data_gemm(const void* dy, const void* w_crsk, void* dx, const sqr_conv_desc* d, const Shape& sh,
                         hipStream_t st) {
  int rc = 0;
  // dX[n,h,w,c] = sum_{r,s,k} dY[n,(h+p-r)/st,(w+p-s)/st,k] W[k,c,r,s] over the divisible taps.
  // Output pixels split by parity (h%st, w%st); in class (ph,pw) only taps r = r0 + st*t contribute
  // and dY row = i + off_h - t: a stride-1 implicit GEMM over the class grid (Hc x Wc).
  const char* wp = (const char*)w_crsk;
  NTArgs cl[4];
  int ncls = 0;
  for (int ph = 0; ph < d->stride; ++ph) {
    for (int pw = 0; pw < d->stride; ++pw) {
      const DgradClass c = dgrad_class(d, ph, pw);
      if (c.Hc == 0 || c.Wc == 0) continue;
      SQR_CHECK_ARG(ncls < 4, "conv2d_bwd_data: stride %d > 2 not supported", d->stride);
      NTArgs& a = cl[ncls++];
      a.g = make_gather(dy, sh.Ho, sh.Wo, d->K, c.Hc, c.Wc, 1, c.off_h, c.off_w, -1, c.Rc > 0 ? c.Rc : 1,
                        c.Sc > 0 ? c.Sc : 1, d->N, sh.ES);
      a.w = wp;
      a.Nout = d->C;
      a.Kg = c.Rc * c.Sc * d->K;  // 0 -> the class receives no gradient: zeros are written
      a.out = dx;
      a.os = d->stride;
      a.stats = nullptr;
      a.oph = ph;
      a.opw = pw;
      a.oH = d->H;
      a.oW = d->W;
      wp += (size_t)d->C * c.Rc * c.Sc * d->K * sh.ES;
    }
  }
  if (ncls == 0) return 0;
  if (d->dtype == SQR_DTYPE_F32) return launch_nt<float>(cl, ncls, st);
  SQR_DISPATCH16(d->dtype, T, rc = launch_nt<T>(cl, ncls, st));
  return rc;
}

static int bwd_weight_impl(const void* x, const void* col_in, const void* dy, float* dw_kcrs,
                           const sqr_conv_desc* d, void* workspace, size_t workspace_bytes, void* stream,
                           const bn::BnFinDev* fin = nullptr, const bn::BnRedDev* red = nullptr,
                           size_t red_lds = 0) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG((x || col_in) && dy && dw_kcrs, "conv2d_bwd_weight: null pointer");
  SQR_CHECK_ARG(!col_in || sh.im2col, "conv2d_bwd_weight_col: only for C<8 (im2col) convs");
  const size_t colb = sh.im2col ? align_up((size_t)sh.M * sh.Kp * sh.ES) : 0;
  const size_t need = sqr_conv2d_workspace_bytes(d, 2) - (col_in ? colb : 0);
  if (!workspace || workspace_bytes < need) {
    set_error("conv2d_bwd_weight: workspace %zu < %zu", workspace_bytes, need);
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  TNArgs a;
  char* ws = (char*)workspace;
  int Ng;
  if (sh.im2col) {
    const void* col = col_in;
    if (!col) {
      if (d->dtype == SQR_DTYPE_F32) rc = im2col<float>(x, d, sh, ws, st);
      else SQR_DISPATCH16(d->dtype, T, rc = im2col<T>(x, d, sh, ws, st));
      if (rc) return rc;
      col = ws;
      ws += colb;
    }
    a.g = make_gather(col, sh.Ho, sh.Wo, sh.Kp, sh.Ho, sh.Wo, 1, 0, 0, 1, 1, 1, d->N, sh.ES);
    Ng = sh.Kp;
  } else {
    a.g = make_gather(x, d->H, d->W, d->C, sh.Ho, sh.Wo, d->stride, -d->pad, -d->pad, 1, d->R, d->S, d->N, sh.ES);
    Ng = d->R * d->S * d->C;
  }
  if (direct3w(d, sh)) {
    int splits = 0;
    const size_t avail = workspace_bytes - (size_t)(ws - (char*)workspace);
    rc = conv3w_launch(d->dtype, x, dy, (float*)ws, avail, d->N, d->H, d->W, d->C, d->K, &splits, st, d->stride);
    if (rc == 0) {
      rc = launch_wgrad_sum((const float*)ws, splits, (long long)d->K * d->C * 9, dw_kcrs, st, fin, red, red_lds);
      if (rc) return rc;
      return 0;
    }
    if (rc != kNotHandled) return rc;
  }
  a.dy = dy;
  a.Kout = d->K;
  a.Ng = Ng;
  a.slab = (float*)ws;
  {
    const int BK = 128 / sh.ES, Wo = a.g.Wo, Ho = a.g.Ho;
    a.rect_wt = 0;
    if (Wo % BK == 0) a.rect_wt = BK;
    else if (BK % Wo == 0 && Ho % (BK / Wo) == 0) a.rect_wt = Wo;
  }
  const TNPlan p = plan_tn(d->K, Ng, sh.M, sh.ES);
  if (d->dtype == SQR_DTYPE_F32) rc = launch_tn<float>(a, p, st);
  else SQR_DISPATCH16(d->dtype, T, rc = launch_tn<T>(a, p, st));
  if (rc) return rc;
  if (!sh.im2col && d->R == 1 && d->S == 1)  // TN slab [K][C] = KCRS
    return launch_wgrad_sum((const float*)ws, p.splits, (long long)d->K * d->C, dw_kcrs, st, fin, red, red_lds);
  return launch_wgrad_reduce((const float*)ws, p.splits, d->K, Ng, d->C, d->R, d->S, sh.im2col ? 1 : d->C,
                             (int)sh.im2col, dw_kcrs, st, fin, red, red_lds);
  return 0;
}

extern "C" int sqr_conv2d_bwd_weight(const void* x, const void* dy, float* dw_kcrs, const sqr_conv_desc* d,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  return bwd_weight_impl(x, nullptr, dy, dw_kcrs, d, workspace, workspace_bytes, stream);
}

extern "C" int sqr_conv2d_bwd_weight_bn(const void* x, const void* dy, float* dw_kcrs, const sqr_conv_desc* d,
                                        const sqr_bn_bwd_fin* fin, const sqr_bn_bwd_red* red, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  bn::BnFinDev f = {};
  if (fin) {
    SQR_CHECK_ARG(fin->stats && fin->stats_rows > 0 && fin->C > 0 && fin->M > 0 && fin->M < (1ll << 31) &&
                      fin->save_mean && fin->save_invstd && fin->coef,
                  "conv2d_bwd_weight_bn: bad BatchNorm finalize job");
    f.part = fin->stats;
    f.nblk = fin->stats_rows;
    f.M = (int)fin->M;
    f.C = fin->C;
    f.gamma = fin->gamma;
    f.mean = fin->save_mean;
    f.invstd = fin->save_invstd;
    f.dgamma = fin->dgamma;
    f.dbeta = fin->dbeta;
    f.coef = fin->coef;
  }
  bn::BnRedDev r = {};
  size_t lds = 0;
  if (red) {
    SQR_CHECK_ARG((red->kind == 1 || red->kind == 2) && red->dy && red->relu_mask && red->x_a && red->mean_a &&
                      (red->kind == 1 || (red->x_b && red->mean_b)) && red->part && red->part_rows,
                  "conv2d_bwd_weight_bn: bad BatchNorm reduction job");
    SQR_CHECK_ARG(red->M > 0 && red->M < (1ll << 31) && red->C >= 8 && red->C <= 2048 && red->C % 8 == 0 &&
                      256 % (red->C / 8) == 0,
                  "conv2d_bwd_weight_bn: bad reduction shape M=%lld C=%d", red->M, red->C);
    r.kind = red->kind;
    r.dtype = d->dtype;
    r.xa = red->x_a;
    r.xb = red->x_b;
    r.dy = red->dy;
    r.mask = red->relu_mask;
    r.mean_a = red->mean_a;
    r.mean_b = red->mean_b;
    r.M = (int)red->M;
    r.C = red->C;
    r.part = red->part;
    bn_red_geometry(red->M, red->C, red->kind, &r.chunk, &r.nblk, &lds);
    *red->part_rows = r.nblk;
  }
  return bwd_weight_impl(x, nullptr, dy, dw_kcrs, d, workspace, workspace_bytes, stream, fin ? &f : nullptr,
                         red ? &r : nullptr, lds);
}

extern "C" int sqr_conv2d_bwd_weight_col(const void* col, const void* dy, float* dw_kcrs, const sqr_conv_desc* d,
                                         void* workspace, size_t workspace_bytes, void* stream) {
  return bwd_weight_impl(nullptr, col, dy, dw_kcrs, d, workspace, workspace_bytes, stream);
}

extern "C" int sqr_conv2d_pack_weights(const sqr_pack_job* jobs, int njobs, void* stream) {
  SQR_CHECK_ARG(jobs && njobs >= 0 && njobs <= 20, "conv2d_pack_weights: 0 <= njobs <= 20 required");
  if (njobs == 0) return 0;
  PackJobs pj;
  int maxtot = 0, maxlds = 0;
  for (int i = 0; i < njobs; ++i) {
    const sqr_conv_desc* d = &jobs[i].desc;
    SQR_CHECK_ARG(jobs[i].w_kcrs && (jobs[i].w_krsc || jobs[i].w_crsk), "conv2d_pack_weights: job %d null", i);
    SQR_CHECK_ARG(d->K >= 1 && d->C >= 1 && d->R >= 1 && d->S >= 1 && d->stride >= 1 && d->stride <= 2 &&
                      d->pad >= 0,
                  "conv2d_pack_weights: job %d bad dims (stride <= 2)", i);
    SQR_CHECK_ARG(d->dtype == SQR_DTYPE_F32 || d->dtype == SQR_DTYPE_BF16 || d->dtype == SQR_DTYPE_F16,
                  "conv2d_pack_weights: bad dtype");
    const int im2col = d->C < 8;
    SQR_CHECK_ARG(!(im2col && jobs[i].w_crsk), "conv2d_pack_weights: no dgrad weights for C<8 convs");
    int kp = 64;
    while (kp < d->R * d->S * d->C) kp *= 2;
    PackJob& j = pj.j[i];
    j.w = jobs[i].w_kcrs;
    j.krsc = jobs[i].w_krsc;
    j.crsk = jobs[i].w_crsk;
    j.K = d->K;
    j.C = d->C;
    j.R = d->R;
    j.S = d->S;
    j.st = d->stride;
    j.pad = d->pad;
    j.im2col = im2col;
    j.Kp = kp;
    j.dtype = d->dtype;
    j.total = d->K * d->C * d->R * d->S;
    j.fd_s = make_fastdiv(d->S);
    j.fd_r = make_fastdiv(d->R);
    j.fd_c = make_fastdiv(d->C);
    int off = 0;
    for (int ph = 0; ph < d->stride; ++ph)
      for (int pw = 0; pw < d->stride; ++pw) {
        const int cl = ph * d->stride + pw;
        const int r0 = (ph + d->pad) % d->stride, s0 = (pw + d->pad) % d->stride;
        const int rc = r0 < d->R ? (d->R - r0 + d->stride - 1) / d->stride : 0;
        const int sc = s0 < d->S ? (d->S - s0 + d->stride - 1) / d->stride : 0;
        j.cls_off[cl] = off;
        j.cls_r0[cl] = r0;
        j.cls_s0[cl] = s0;
        j.cls_rc[cl] = rc;
        j.cls_sc[cl] = sc;
        off += d->C * rc * sc * d->K;
      }
    const int rows = d->K > d->C ? d->K : d->C;
    maxtot = rows > maxtot ? rows : maxtot;
    const int lds = (d->K > d->C ? d->K : d->C) * d->R * d->S;
    maxlds = lds > maxlds ? lds : maxlds;
  }
  SQR_CHECK_ARG(maxlds * 4 <= 160 * 1024, "conv2d_pack_weights: weight rows too large for LDS staging");
  hipLaunchKernelGGL(pack_weights_batched_kernel, dim3(maxtot, njobs, 2), dim3(256), (size_t)maxlds * 4,
                     as_stream(stream), pj);
  SQR_HIP_LAUNCH_CHECK("pack_weights_batched_kernel");
  return 0;
}
