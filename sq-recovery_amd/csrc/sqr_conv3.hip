// Direct 3x3 / stride 1 / pad 1 convolution (forward and backward-data), bf16 / fp16, gfx950 MFMA.
//
// The generic implicit-GEMM kernel (sqr_conv.hip conv_nt_kernel) gathers every (pixel, tap) row
// of the im2col matrix separately: per 64-channel k-tile it pays one LDS-DMA piece per 8 rows
// plus the per-row bounds/address VALU, 9 times over the same input pixels, and measured
// 7.4 VALU per MFMA on the layer-1 shape (PMC, profiles/).  Here a workgroup owns a TH x TW
// pixel rectangle of one image and stages its (TH+2) x (TW+2) halo window ONCE per 64-channel
// chunk; the 9 taps are then 9 shifted views of that window (a per-tap uniform row offset), so
// per k-step only the BN x 64 weight tile streams in, through a buffer-descriptor LDS-DMA ring
// whose per-step offsets are scalar (soffset) — no per-row address VALU in the loop at all.
//
//   out[p][n] = sum_{tap, c} win[p + shift(tap)][c] * Wt[n][tap][c]
//   forward:       win = X,  Wt = w_krsc [K][3][3][C],  shift(r,s) = (r, s)
//   backward-data: win = dY, Wt = w_crsk [C][3][3][K],  shift(r,s) = (2-r, 2-s)   (flip)
//
// LDS rows are 128 B (64 bf16 channels) with a 16-B slot XOR swizzle slot ^ (row & 6) (d3key):
// for ANY 16 consecutive rows -- whatever the tap shift -- the ds_read_b128 fragment reads
// (lanes fr = row offset 0..15, fq = slot) hit 16 distinct bank quads in every lane group.  (The
// NT kernel's key (row>>1)&7 is conflict-free only for 16-aligned row groups: 2-way on 2/3 taps.)  Halo / out-of-image pixels come back as zeros from the
// buffer descriptor range check (voffset = 0x80000000).
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>
#include "sqr_conv_dev.h"

namespace sqr {
namespace conv {

// SQR_STAMPS builds (tools/conv_stamps.py, never the shipped library): a kernel whose clock probe is
// armed keeps five wall-clock stamps per workgroup (start, prologue done, first chunk done, main loop
// done, stores drained) and writes them to tp[2 + 8 * blockIdx.x ...] at its end, beside blockIdx.x.
// The buffer holds SQR_STAMP_MAXWG workgroups (tools/conv_stamps.py sizes it from the same number);
// workgroups past it keep no stamps.
#ifdef SQR_STAMPS
#ifndef SQR_STAMP_MAXWG
#define SQR_STAMP_MAXWG 8192
#endif
#define SQR_STAMP_DECL unsigned long long stamp_[5] = {0, 0, 0, 0, 0};
#define SQR_STAMP(i) (stamp_[i] = wall_clock64())
#define SQR_STAMP_WRITE(tp)                                                              \
  do {                                                                                   \
    if ((tp) && threadIdx.x == 0 && blockIdx.x < SQR_STAMP_MAXWG) {                      \
      for (int i_ = 0; i_ < 5; ++i_) (tp)[2 + 8 * blockIdx.x + i_] = stamp_[i_];          \
      (tp)[2 + 8 * blockIdx.x + 5] = blockIdx.x;                                         \
    }                                                                                    \
  } while (0)
#else
#define SQR_STAMP_DECL
#define SQR_STAMP(i) ((void)0)
#define SQR_STAMP_WRITE(tp) ((void)0)
#endif

// 16-B slot XOR key of a 128-B LDS row (see the header): shift-invariant conflict-free b128 reads
__device__ __forceinline__ int d3key(int row) { return row & 6; }

// Window key of 8-pixel-wide tiles (TW = 8, window rows WWID = 10 pixels): a fragment's 16 pixels
// are two runs of 8 window rows, 10 apart, which row & 6 serves 2-way conflicted (the runs' rows
// share parity and key).  Key of row r = entry r % 20 of a 20-entry table (3 bits each), found by
// search over every fragment read the kernel makes (tap offsets r*10 + c, pixel rows y even, both
// images of a two-image tile, flipped taps): every ds_read_b128 lane group hits 16 distinct bank
// quads.
constexpr unsigned long long K20_LUT = 0xadc1f8859b07e93ull;
__device__ __forceinline__ int k20key(int row) { return (int)((K20_LUT >> (3 * (row % 20))) & 7); }

struct D3Args {
  const void* x;    // [N][H][W][Cin]
  const void* w;    // [Nout][9][Cin]
  void* out;        // [N][H][W][Nout]
  const void* addend;  // nullable: out = conv + addend ([N][H][W][Nout], may alias out)
  const uint8_t* addend_mask;  // nullable (ACC): the addend counts only where its bit is set (1 bit / element)
  const void* bn_x;        // BNB: the following BatchNorm's input [N][H][W][Nout], its ReLU mask and
  const uint8_t* bn_mask;  //      batch mean: out = conv * mask, stats = (sum g, sum g*(x - mean))
  const float* bn_mean;
  const float* bn_coef;  // BNB, nullable: the mask is recomputed from bn_x and the BatchNorm's forward
                         // [2][Nout] (scale, shift) instead of read from bn_mask ...
  void* bn_act;          // ... and, if set, the activation relu(bn_x * scale + shift) is written here
  const float* in_coef;  // BNIN: [2][Cin] (scale, shift) of the preceding BatchNorm + ReLU, applied on load
  float* stats;     // nullable: BatchNorm partials [ntm][2][Nout]
  int N, H, W, Cin, Nout;  // H, W: the OUTPUT size
  int iH, iW;              // the input size (= H, W at stride 1; 2H, 2W at stride 2)
  int tiles_x, tiles_per_img;
  int ntm, ntn;
  int flip;
  uint32_t xbytes, wbytes;
  unsigned long long* tp;  // nullable: clock probe slots
#ifdef SQR_EXPERIMENTS
  int exp;  // ablation bits (experiment builds only, tools/build_exp.sh): 2 no output stores, 4 no MFMAs,
            // 8 no in-loop weight DMA (wrong results: timing only)
#endif
};

// SQR_EXPERIMENTS builds: ablation bit test (always false in the shipped library)
#ifdef SQR_EXPERIMENTS
#define SQR_ABL(a, bit) (((a).exp & (bit)) != 0)
#else
#define SQR_ABL(a, bit) false
#endif

// one 1-KiB LDS-DMA piece (16 B per lane to dst + 16*lane)
__device__ __forceinline__ void dma_piece(__amdgpu_buffer_rsrc_t srd, char* dst, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(srd, (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
}

// LDS-DMA issue of PIECES 1-KiB pieces per wave: piece i of wave w lands at rows
// (i*NW + w)*8 .. +7 of dst; per-lane voffsets are fixed, the scalar soffset selects chunk / tap
template <int PIECES, int NW>
__device__ __forceinline__ void dma_pieces(__amdgpu_buffer_rsrc_t srd, char* dst, const uint32_t* voff, int soff,
                                           int wave) {
#pragma unroll
  for (int i = 0; i < PIECES; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(srd, (__attribute__((address_space(3))) void*)(dst + ((i * NW + wave) * 8) * 128),
                                             16, voff[i], soff, 0, 0);
}

// Backward sums of a BM x BN output tile (BNB: sum g, sum g*(x - mean)) held as per-lane partials
// s1, s2 (lane: pixel 16i+fr of its wave rows, channels 16j+4fq..+3 of its wave columns): an LDS
// transpose red[wave-row group][fr][col], then one thread per column adds its 16*WAVES_M partials
// in a fixed order (deterministic, no cross-lane shuffles).
template <int BN, int WAVES_M, int WAVES_N, int TN, int NT>
__device__ __forceinline__ void stats_reduce(const float (*s1)[4], const float (*s2)[4], float* red, int wm, int wn,
                                             int fr, int fq, int tid, float* stats_row0, float* stats_row1) {
  constexpr int WN = BN / WAVES_N;
  // red: [2][WAVES_M*16 rows][BN cols] floats
  float* r1 = red + (wm * 16 + fr) * BN + wn * WN + 4 * fq;
  float* r2 = r1 + WAVES_M * 16 * BN;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    *(f32x4*)(r1 + 16 * j) = f32x4{s1[j][0], s1[j][1], s1[j][2], s1[j][3]};
    *(f32x4*)(r2 + 16 * j) = f32x4{s2[j][0], s2[j][1], s2[j][2], s2[j][3]};
  }
  __syncthreads();
  for (int c = tid; c < 2 * BN; c += NT) {
    const int q = c / BN, col = c - q * BN;
    const float* src = red + q * WAVES_M * 16 * BN + col;
    float acc = 0.f;
#pragma unroll 8
    for (int r = 0; r < WAVES_M * 16; ++r) acc += src[r * BN];
    (q ? stats_row1 : stats_row0)[col] = acc;
  }
}

// Forward BatchNorm statistics of a BM x BN output tile held as acc[j][i], from the 16-bit values
// actually stored: the tile's Welford row (mean, M2) per channel.  The 16 lanes of a quarter-wave
// (same fq: the same 4 channels, 16 pixel rows of TM values each) shift by the group's first value K
// (lane fr = 0, value 0: broadcast), add their shifted values and squares as plain floats over an xor
// tree and leave (mean = K + S/n, M2 = Q - S^2/n) for n = 16 TM values — no cancellation while the
// values stay within a few std of K, no per-level division; the WAVES_M group rows of a column are
// merged by one thread in a fixed order (lane_rows_merge, float64).  Row count BM (written once per
// tile row by the tile_n = 0 workgroup).
template <typename T, int BN, int WAVES_M, int WAVES_N, int TM, int TN, int NT>
__device__ __forceinline__ void tile_stats(const uint32_t (*pk)[TM][2], float* red, int wm, int wn, int fr, int fq,
                                           int tid, float* stats_row0, float* stats_row1, float* count, float bm) {
  constexpr int WN = BN / WAVES_N;
  constexpr float NG = 16.f * TM, INV_NG = 1.f / (16.f * TM);
  float* r1 = red + wm * BN + wn * WN + 4 * fq;
  float* r2 = r1 + WAVES_M * BN;
  // all TN * 4 channel chains first, then one guarded write: a write per j inside the loop split the
  // chains into TN serial groups (an exec-masked branch between them)
  float m[TN][4], q[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) v[i] = (e & 1) ? hi2f<T>(pk[j][i][e >> 1]) : lo2f<T>(pk[j][i][e >> 1]);
      const float K = row_first(v[0]);  // lane fr = 0 of the 16-lane row (DPP broadcast, no LDS)
      float sa = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float d = v[i] - K;
        sa += d;
        sq = fmaf(d, d, sq);
      }
      // DPP row sums (four row_shr adds each, totals in lane fr = 15) instead of four ds_bpermute
      // levels per value: the epilogue's 8 * TN * 4 dependent LDS round trips were most of its time
      sa = row_sum15(sa);
      sq = row_sum15(sq);
      const float sn = sa * INV_NG;
      m[j][e] = K + sn;
      q[j][e] = fmaxf(sq - sa * sn, 0.f);
    }
  }
  if (fr == 15) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      *(f32x4*)(r1 + 16 * j) = f32x4{m[j][0], m[j][1], m[j][2], m[j][3]};
      *(f32x4*)(r2 + 16 * j) = f32x4{q[j][0], q[j][1], q[j][2], q[j][3]};
    }
  }
  __syncthreads();
  for (int col = tid; col < BN; col += NT) {
    float mean, m2;
    lane_rows_merge(red + col, red + WAVES_M * BN + col, WAVES_M, BN, NG, &mean, &m2);
    stats_row0[col] = mean;
    stats_row1[col] = m2;
  }
  if (count && tid == 0) *count = bm;
}

// IMGS > 1: a tile is IMGS whole images (TH x TW = H x W) with one halo window each, stacked in LDS
// (small late-layer images: more pixels per weight tile fetched)
// PD: weight tiles prefetched ahead (ring of PD + 1 stages): the per-CU LDS-DMA delivery is
// latency x bytes-in-flight bound, so deeper rings buy throughput where LDS allows
// ACC (backward-data of a block input): out = conv + a.addend.  The addend is loaded into registers
// before the first DMA of the kernel, so its HBM read overlaps the main loop instead of adding a
// burst at the end (measured at B=64: +3.9 us on layer 2 when read in the epilogue).
// BNB (backward-data into a BatchNorm+ReLU backward): x and the mask bits at the lane's outputs are
// loaded before the main loop like ACC's addend; the stored value is g = conv * mask and the tile's
// partial row of a.stats gets the BatchNorm backward sums (sum g, sum g*(x - mean)).  With a.bn_coef
// the mask is not read: it is recomputed from x and the BatchNorm's forward (scale, shift) exactly as
// the apply pass forms it (the rounded activation > 0), and the activation itself can be written
// (a.bn_act: the weight gradient's input, never stored by the forward -- BNIN below).
// BNIN (forward, stride 1): the input x is the PRE-activation of a BatchNorm + ReLU whose (scale,
// shift) are a.in_coef: each chunk's halo window is transformed in LDS to relu(x * scale + shift),
// bitwise what the apply pass writes, after it lands and before anyone reads it -- every lane rewrites
// the 16-B pieces its own LDS-DMA fetched (padding pieces stay zero: the conv pads the activation).
// A lane's pieces all hold the same 8 channels of a chunk (slot pslot ^ (prow & 6); hence no K20
// window key): its 16 coefficients of a chunk are 4 LDS reads from a [2][Cin] table staged in the
// prologue (no global load inside the loop: a compiler-tracked load there made the compiler drain
// every in-flight weight tile before its first use).
// S = 2 (forward of a 3x3 / stride-2 / pad-1 conv, IMGS = 1, no flip): the (2TH+1) x (2TW+1) input
// window of a TH x TW output tile is staged as four phase planes (a, b) = (input row, column parity
// relative to the window origin), each TW+1 pixels wide (plane (., 1) has one unused column), plane
// (a, .) holding TH+1-a rows.  Tap (r, c) of output pixel (y, x) reads plane (r & 1, c & 1) at
// (y + (r >> 1), x + (c >> 1)): consecutive output pixels are consecutive plane rows and the tap
// offset is one constant per tap, so the stride-1 fragment reads carry over unchanged.
// SQR_D3_WINPF: read the next tap's first window fragments before each step's barrier
#ifndef SQR_D3_WINPF
#define SQR_D3_WINPF 1
#endif
template <typename T, int BM, int BN, int WAVES_M, int WAVES_N, int TW, int TH, int NWB, int IMGS = 1, int PD = 2,
          bool ACC = false, bool BNB = false, int S = 1, bool BNIN = false>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N) conv3_kernel(D3Args a) {
  constexpr int NT = 64 * WAVES_M * WAVES_N, NW = WAVES_M * WAVES_N;
  constexpr int ROWB = 128, STAGES = PD + 1;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert(S == 1 || (S == 2 && IMGS == 1 && !ACC && !BNB), "stride 2: forward, one image per tile");
  constexpr int WWID = S == 1 ? TW + 2 : TW + 1;
  static_assert(!BNIN || (S == 1 && !ACC && !BNB), "apply-on-load: stride-1 forward");
  constexpr bool K20 = S == 1 && TW == 8 && !BNIN;  // window rows keyed by k20key (8-pixel-wide tiles)
  constexpr int P0 = (TH + 1) * WWID, P1 = TH * WWID;  // stride 2: rows of an a = 0 / a = 1 plane
  constexpr int WRI = S == 1 ? (TH + 2) * WWID : 2 * P0 + 2 * P1, WR = IMGS * WRI;  // halo window rows
  constexpr int WROWS = (WR + 8 * NW - 1) / (8 * NW) * (8 * NW);
  constexpr int PB = BN / (8 * NW);                          // weight pieces per wave per step
  constexpr int WP = WROWS / (8 * NW);                       // window pieces per wave per chunk
  static_assert(BM == IMGS * TH * TW, "pixel tile");
  static_assert(PB >= 1 && PB * 8 * NW == BN, "BN must be a multiple of 8 * waves");
  constexpr int WIN = WROWS * ROWB, TILE_B = BN * ROWB;
  constexpr int LDS = NWB * WIN + STAGES * TILE_B;
  static_assert(2 * WAVES_M * 16 * BN * 4 <= LDS, "stats scratch fits the ring");
  // BNIN: the coefficient table [scale Cin][shift Cin] after the ring, in the same LDS array (a second
  // __shared__ object made the compiler wait for every in-flight LDS-DMA before each window read)
  __shared__ __attribute__((aligned(1024))) char smem[LDS + (BNIN ? 2 * 512 * 4 : 0)];
  float* const ctab = (float*)(smem + LDS);
  char* const bring = smem + NWB * WIN;
  clock_begin(a.tp);
  SQR_STAMP_DECL
  SQR_STAMP(0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_m = bid / a.ntn, tile_n = bid - (bid / a.ntn) * a.ntn;
  const int img = (tile_m / a.tiles_per_img) * IMGS;  // first image of the tile
  const int trem = tile_m - (tile_m / a.tiles_per_img) * a.tiles_per_img;
  const int ty = trem / a.tiles_x, tx = trem - ty * a.tiles_x;
  const int h0 = ty * TH, w0 = tx * TW, n0 = tile_n * BN;

  // output element offset of this lane's pixel i, channels n0 + wn*WN + 4fq (+ 16 j)
  const int fr = lane & 15, fq = lane >> 4;
  auto out_off = [&](int i) -> size_t {
    const int m = wm * WM + 16 * i + fr;
    const int ii = m / (TH * TW), mm = m - ii * (TH * TW);
    return (((size_t)(img + ii) * a.H + h0 + mm / TW) * a.W + w0 + (mm % TW)) * a.Nout + n0 + wn * WN + 4 * fq;
  };
  u32x2 av[ACC || BNB ? TN : 1][ACC || BNB ? TM : 1];
  uint32_t bmk[(BNB || ACC) ? TN : 1][(BNB || ACC) ? TM : 1];
  // LATE: 4-wave workgroups with 64 x 64 wave tiles (TM * TN >= 16) load the addend / BatchNorm
  // operands in the epilogue instead of holding them through the main loop: held, they take the
  // kernel past 256 VGPRs and halve its occupancy from two workgroups per CU to one (config 5's
  // 128x128 layer-1 dgrad + addend: 118 -> 178 us).  8-wave workgroups run one per CU either way
  // and keep the early load (its latency hides behind the main loop).
  constexpr bool LATE = NW == 4 && TM * TN >= 16;
  auto load_av = [&]() {
    const uint16_t* ad = (const uint16_t*)(BNB ? a.bn_x : a.addend);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const size_t o = out_off(i);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        av[j][i] = *(const u32x2*)(ad + o + 16 * j);
        if constexpr (BNB) bmk[j][i] = a.bn_coef ? 0u : a.bn_mask[(o + 16 * j) >> 3];
        if constexpr (ACC) bmk[j][i] = a.addend_mask ? a.addend_mask[(o + 16 * j) >> 3] : 0xffu;
      }
    }
  };
  if constexpr ((ACC || BNB) && !LATE) load_av();

  // ---- per-lane DMA offsets (fixed for the whole kernel; chunk / tap parts are scalar)
  constexpr uint32_t kOOB = 0x80000000u;
  const int prow = lane >> 3, pslot = lane & 7;
  uint32_t wvoff[WP];
#pragma unroll
  for (int i = 0; i < WP; ++i) {
    const int r = (i * NW + wave) * 8 + prow;  // window row
    const int ls = pslot ^ (K20 ? k20key(r) : d3key(r));  // logical 16-B channel slot this lane fetches
    const int ii = r / WRI, rr = r - ii * WRI;     // image of the tile, row in its window
    int h, w;
    bool used = r < WR;
    if constexpr (S == 1) {
      const int wy = rr / WWID, wx = rr - wy * WWID;  // constant divisors
      h = h0 - 1 + wy;
      w = w0 - 1 + wx;
    } else {  // plane (pa, pb) row (py, px) <- input (2h0 - 1 + 2py + pa, 2w0 - 1 + 2px + pb)
      const int pa = rr >= 2 * P0 ? 1 : 0;
      const int pb = pa ? (rr >= 2 * P0 + P1 ? 1 : 0) : (rr >= P0 ? 1 : 0);
      const int pr = rr - (pa ? 2 * P0 + pb * P1 : pb * P0);
      const int py = pr / WWID, px = pr - py * WWID;
      h = 2 * h0 - 1 + 2 * py + pa;
      w = 2 * w0 - 1 + 2 * px + pb;
      used = used && (pb == 0 || px < TW);
    }
    const bool ok = used && (unsigned)h < (unsigned)a.iH && (unsigned)w < (unsigned)a.iW;
    wvoff[i] = ok ? (uint32_t)(((((img + ii) * a.iH + h) * a.iW + w) * a.Cin) * 2 + ls * 16) : kOOB;
  }
  uint32_t bvoff[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int r = (i * NW + wave) * 8 + prow;  // weight row = output channel n0 + r
    const int ls = pslot ^ d3key(r);
    bvoff[i] = (uint32_t)(((n0 + r) * 9 * a.Cin) * 2 + ls * 16);
  }
  const __amdgpu_buffer_rsrc_t xsrd = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsrd = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, a.wbytes, 0x00020000);

  // ---- fragment coordinates
  int qbase[TM];  // window row of this lane's output pixel at tap shift (0, 0)
  // K20: the window keys of row qbase + toff for the 6 tap offsets mod 20 (c + 10 b, b < 2, c < 3),
  // 3 bits each
  int qkey[K20 ? TM : 1];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wm * WM + 16 * i + fr;
    const int ii = m / (TH * TW), mm = m - ii * (TH * TW);
    qbase[i] = ii * WRI + (mm / TW) * WWID + (mm % TW);
    if constexpr (K20) {
      int kk = 0;
#pragma unroll
      for (int j = 0; j < 6; ++j) kk |= k20key(qbase[i] + (j % 3) + 10 * (j / 3)) << (3 * j);
      qkey[i] = kk;
    }
  }
  int poff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int row = wn * WN + 16 * j + fr;
    poff[j] = row * ROWB + ((fq ^ d3key(row)) << 4);  // slot fq; sub 1 = slot fq+4 = ^ 64 B
  }

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = a.Cin >> 6;
  const int flip = a.flip;
  const int nsteps = nch * 9;
  // NWB = 1: one window buffer, never reloaded -- Cin = 64 (one chunk) only (pick / pick_s2f)
  constexpr int WPN = NWB == 2 ? WP : 0;  // window pieces a deep-ring step issues at tap 0
  static_assert(PB * (PD - 1) + WP <= 63, "vmcnt range");
  static_assert(PD >= 2 && PD <= 8, "the next window must be older than the tile retired at tap 8");
  // weight tile of global step q = 9 * chunk + tap (clamped: the dummy reloads past the end keep
  // every wave's count of loads in flight uniform, and land in slots nobody reads again)
  auto issue_w = [&](int q) {
    q = q < nsteps ? q : nsteps - 1;
    const int cq = q / 9, tq = q - cq * 9;
    dma_pieces<PB, NW>(wsrd, bring + ((q % STAGES) * TILE_B), bvoff,
                       __builtin_amdgcn_readfirstlane((tq * a.Cin + cq * 64) * 2), wave);
  };
  // BNIN: this lane's 8 channels of a chunk (slot lslot) and their (scale, shift); the window pieces a
  // lane fetched are rewritten in place once landed (bn_in_window), padding pieces left zero
  const int lslot = pslot ^ (prow & 6);
  // the coefficient table (2 Cin <= 4 NT floats: one 16-B load per thread, issued before the prologue's
  // DMA and written to LDS after it, so the load's latency overlaps the DMA's)
  static_assert(!BNIN || 2 * 512 <= 4 * NT, "coefficient table: one load per thread");
  f32x4 ctv = {0.f, 0.f, 0.f, 0.f};
  if constexpr (BNIN) {
    if (tid < a.Cin / 2) ctv = *(const f32x4*)(a.in_coef + 4 * tid);
  }
  f32x4 icf[BNIN ? 4 : 1];
  auto load_icoef = [&](int ch) {
    if constexpr (BNIN) {
      const float* c = ctab + ch * 64 + lslot * 8;
      icf[0] = *(const f32x4*)c;
      icf[1] = *(const f32x4*)(c + 4);
      icf[2] = *(const f32x4*)(c + a.Cin);
      icf[3] = *(const f32x4*)(c + a.Cin + 4);
    }
  };
  auto bn_in_window = [&](char* wbuf) {
    if constexpr (BNIN) {
#pragma unroll
      for (int i = 0; i < WP; ++i) {
        if (wvoff[i] != kOOB) {
          u32x4* pp = (u32x4*)(wbuf + ((i * NW + wave) * 8) * ROWB + lane * 16);
          u32x4 v = *pp;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float sc0 = icf[e >> 1][2 * (e & 1)], sc1 = icf[e >> 1][2 * (e & 1) + 1];
            const float sh0 = icf[2 + (e >> 1)][2 * (e & 1)], sh1 = icf[2 + (e >> 1)][2 * (e & 1) + 1];
            v[e] = pack2<T>(fmaxf(fmaf(lo2f<T>(v[e]), sc0, sh0), 0.f), fmaxf(fmaf(hi2f<T>(v[e]), sc1, sh1), 0.f));
          }
          *pp = v;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  dma_pieces<WP, NW>(xsrd, smem, wvoff, 0, wave);
#pragma unroll
  for (int q = 0; q < PD; ++q) issue_w(q);
  // window 0 and weight tile 0 landed; tiles 1 .. PD-1 stay in flight
  if constexpr (PD == 2) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PB) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PB * (PD - 1)) : "memory");
  }
  if constexpr (BNIN) {
    if (tid < a.Cin / 2) *(f32x4*)(ctab + 4 * tid) = ctv;
    __syncthreads();  // the coefficient table
    load_icoef(0);
    bn_in_window(smem);
  }
  __builtin_amdgcn_s_barrier();
  SQR_STAMP(1);

  // window fragment offsets of tap t (r, c3) for this lane's TM pixel rows
  auto tap_qoff = [&](int t, int* qo) {
    const int r = t / 3, c3 = t % 3;
    int toff;
    if constexpr (S == 1) {
      toff = flip ? (2 - r) * WWID + (2 - c3) : r * WWID + c3;
    } else {
      toff = ((r & 1) ? 2 * P0 + (c3 & 1) * P1 : (c3 & 1) * P0) + (r >> 1) * WWID + (c3 >> 1);
    }
    // K20: tap offset toff = 10 r' + c' (r', c' the possibly flipped tap) is 10 (r' & 1) + c' mod 20
    const int kj = K20 ? 3 * ((flip ? 2 - c3 : c3) + 3 * ((flip ? 2 - r : r) & 1)) : 0;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int row = qbase[i] + toff;
      // keep the per-tap address math here: hoisted for all 9 unrolled taps it spills
      asm volatile("" : "+v"(row));
      const int key = K20 ? (qkey[i] >> kj) & 7 : d3key(row);
      qo[i] = row * ROWB + ((fq ^ key) << 4);
    }
  };
  constexpr bool kWinPrefetch = SQR_D3_WINPF;
  int qoff_n[TM];
  V8<T> qn[TM];

  for (int cc = 0; cc < nch; ++cc) {
    const bool next = cc + 1 < nch;
    const char* win = smem + (NWB == 2 ? (cc & 1) * WIN : 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int step = cc * 9 + t;
      // this step's LDS-DMA issue (the weight tile PD steps ahead, at tap 0 the next chunk's window),
      // placed after the step's MFMAs: issued among them it costs the waves more issue cycles
      // (same-box kernel timings: 0.3-0.8 us less per launch on layers 2-3, 1.4 % over the nine
      // tiled shapes, profiles/r04dp_tiled_conv_dma_position.jsonl)
      auto issue_step = [&]() {
        if constexpr (PD == 2) {
          // (the original 3-stage schedule: no loads past the end)
          if (t < 7) {
            dma_pieces<PB, NW>(wsrd, bring + ((t + 2) % 3) * TILE_B, bvoff,
                               __builtin_amdgcn_readfirstlane(((t + 2) * a.Cin + cc * 64) * 2), wave);
          } else if (next) {
            dma_pieces<PB, NW>(wsrd, bring + ((t + 2) % 3) * TILE_B, bvoff,
                               __builtin_amdgcn_readfirstlane(((t - 7) * a.Cin + (cc + 1) * 64) * 2), wave);
          }
          if (NWB == 2 && t == 0 && next)
            dma_pieces<WP, NW>(xsrd, smem + ((cc + 1) & 1) * WIN, wvoff, __builtin_amdgcn_readfirstlane((cc + 1) * 128),
                               wave);
        } else {
          issue_w(step + PD);
          if (NWB == 2 && t == 0)  // next chunk's window (the last chunk reloads its own into the idle buffer)
            dma_pieces<WP, NW>(xsrd, smem + ((cc + 1) & 1) * WIN, wvoff,
                               __builtin_amdgcn_readfirstlane((next ? cc + 1 : cc) * 128), wave);
        }
      };
      const char* bst = bring + (PD == 2 ? (t % 3) : (step % STAGES)) * TILE_B;
      int qoff[TM];
      if constexpr (kWinPrefetch) {
        if (t == 0) tap_qoff(0, qoff);
#pragma unroll
        for (int i = 0; i < TM; ++i)
          if (t > 0) qoff[i] = qoff_n[i];
      } else {
        tap_qoff(t, qoff);
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        V8<T> pf[TN], qf[TM];
#pragma unroll
        for (int j = 0; j < TN; ++j) pf[j] = *(const V8<T>*)(bst + (poff[j] ^ (sub << 6)));
#pragma unroll
        for (int i = 0; i < TM; ++i)
          qf[i] = kWinPrefetch && sub == 0 && t > 0 ? qn[i] : *(const V8<T>*)(win + (qoff[i] ^ (sub << 6)));
        if (SQR_ABL(a, 4)) {
#pragma unroll
          for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(pf[j]));
#pragma unroll
          for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(qf[i]));
        } else {
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
        }
      }
      if (!SQR_ABL(a, 8) || t == 0) issue_step();
      // the next tap's first window fragments, read before this step's barrier: the window of a
      // chunk is stable through its 9 taps (only the weight stage needs the barrier), so after it
      // only the weight fragments' LDS latency stands between the barrier and the first MFMA
      if constexpr (kWinPrefetch) {
        if (t < 8) {
          tap_qoff(t + 1, qoff_n);
#pragma unroll
          for (int i = 0; i < TM; ++i) qn[i] = *(const V8<T>*)(win + qoff_n[i]);
        }
      }
      // the window prefetch (TM reads, the youngest LDS operations) stays in flight over the barrier
      const bool pre = kWinPrefetch && t < 8;
      // Every step-end wait also retires this wave's own LDS reads (lgkmcnt(0)): the raw s_barrier
      // does not wait for them on gfx950, and after it other waves DMA into the stage just read —
      // an LDS-DMA write is not ordered behind another wave's queued ds_read, so a read still in
      // the LDS queue could see the next tile (seen as a rare wrong 16-channel fragment at B = 16
      // with two workgroups per CU; the epilogue's reuse of the LDS for statistics relies on it too)
#define SQR_D3_STEP_WAIT(V)                                                                  \
  do {                                                                                       \
    if (pre)                                                                                 \
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(%1)" ::"n"(V), "n"(TM) : "memory");          \
    else                                                                                     \
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(V) : "memory");                     \
  } while (0)
      if constexpr (PD == 2) {
        const bool more = t < 7 || next;
        // retire the weight tile of the next step (and at tap 8 the next window, which is older);
        // at taps 0-1 the next chunk's window is younger than it and stays in flight
        if (!more) {
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        } else if (NWB == 2 && t <= 1 && next) {
          SQR_D3_STEP_WAIT(PB + WP);
        } else {
          SQR_D3_STEP_WAIT(PB);
        }
      } else {
        // retire weight tile step+1 (issued at step+1-PD): younger are tiles step+2 .. step+PD and,
        // for t <= PD-1, this chunk's window load (issued at t = 0 after that step's tile load)
        if (t <= PD - 1) {
          SQR_D3_STEP_WAIT(PB * (PD - 1) + WPN);
        } else {
          SQR_D3_STEP_WAIT(PB * (PD - 1));
        }
      }
#undef SQR_D3_STEP_WAIT
      // the next chunk's window has landed (the step-end wait of tap 8 retires it): BatchNorm + ReLU
      // applied in place before the barrier that publishes it
      if (BNIN && t == 8 && next) {
        load_icoef(cc + 1);
        bn_in_window(smem + ((cc + 1) & 1) * WIN);
      }
      __builtin_amdgcn_s_barrier();
    }
    if (cc == 0) SQR_STAMP(2);
  }
  SQR_STAMP(3);
  if constexpr (PD != 2) {  // drain the dummy loads before the epilogue reuses the LDS
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue: lane holds out[pixel m][n..n+3]; convert once (ACC: after adding the addend),
  // store, then BN partials
  size_t opix[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) opix[i] = out_off(i);
  if constexpr ((ACC || BNB) && LATE) load_av();
  if constexpr (ACC) {  // (a masked addend: cleared halves are +0, as the masked tensor would hold)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const uint32_t mb = (bmk[j][i] >> ((opix[i] + 16 * j) & 4)) & 0xfu;
        const uint32_t a0 = av[j][i][0] & (((mb & 1u) ? 0xffffu : 0u) | ((mb & 2u) ? 0xffff0000u : 0u));
        const uint32_t a1 = av[j][i][1] & (((mb & 4u) ? 0xffffu : 0u) | ((mb & 8u) ? 0xffff0000u : 0u));
        acc[j][i][0] += lo2f<T>(a0);
        acc[j][i][1] += hi2f<T>(a0);
        acc[j][i][2] += lo2f<T>(a1);
        acc[j][i][3] += hi2f<T>(a1);
      }
  }
  uint32_t pk[TN][TM][2];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      pk[j][i][0] = pack2<T>(acc[j][i][0], acc[j][i][1]);
      pk[j][i][1] = pack2<T>(acc[j][i][2], acc[j][i][3]);
    }
  // BNB with a.bn_coef: the lane's activation relu(x * scale + shift) (packed as the apply pass packs
  // it) and its ReLU mask, from x and the BatchNorm's forward coefficients
  uint32_t ak[BNB ? TN : 1][BNB ? TM : 1][2];
  if constexpr (BNB) {  // g = conv * mask (4 channels of the lane: mask bits (opix & 4) .. +3)
    const bool bc = a.bn_coef != nullptr;
    float s1[TN][4], s2[TN][4], mu[TN][4], csc[TN][4], csh[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = n0 + wn * WN + 16 * j + 4 * fq + e;
        s1[j][e] = s2[j][e] = 0.f;
        mu[j][e] = a.bn_mean[c];
        // (loads from a selected valid pointer: no load behind the null test)
        const float* cp = bc ? a.bn_coef : a.bn_mean;
        csc[j][e] = cp[c];
        csh[j][e] = cp[bc ? a.Nout + c : c];
      }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        uint32_t mb;
        if (bc) {
          mb = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t v = pack2<T>(fmaxf(fmaf(lo2f<T>(av[j][i][h]), csc[j][2 * h], csh[j][2 * h]), 0.f),
                                        fmaxf(fmaf(hi2f<T>(av[j][i][h]), csc[j][2 * h + 1], csh[j][2 * h + 1]), 0.f));
            ak[j][i][h] = v;
            mb |= (lo2f<T>(v) > 0.f ? 1u : 0u) << (2 * h);
            mb |= (hi2f<T>(v) > 0.f ? 1u : 0u) << (2 * h + 1);
          }
        } else {
          mb = (bmk[j][i] >> ((opix[i] + 16 * j) & 4)) & 0xfu;
        }
        pk[j][i][0] &= ((mb & 1u) ? 0xffffu : 0u) | ((mb & 2u) ? 0xffff0000u : 0u);
        pk[j][i][1] &= ((mb & 4u) ? 0xffffu : 0u) | ((mb & 8u) ? 0xffff0000u : 0u);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float g0 = lo2f<T>(pk[j][i][h]), g1 = hi2f<T>(pk[j][i][h]);
          s1[j][2 * h] += g0;
          s2[j][2 * h] = fmaf(g0, lo2f<T>(av[j][i][h]) - mu[j][2 * h], s2[j][2 * h]);
          s1[j][2 * h + 1] += g1;
          s2[j][2 * h + 1] = fmaf(g1, hi2f<T>(av[j][i][h]) - mu[j][2 * h + 1], s2[j][2 * h + 1]);
        }
      }
    stats_reduce<BN, WAVES_M, WAVES_N, TN, NT>(s1, s2, (float*)smem, wm, wn, fr, fq, tid,
                                               a.stats + ((size_t)tile_m * 2) * a.Nout + n0,
                                               a.stats + ((size_t)tile_m * 2 + 1) * a.Nout + n0);
  }
  uint16_t* out = (uint16_t*)a.out;
  // 16-B stores: a lane holds 4 channels (8 B) of each 16-channel tile j; v_permlane16_swap of the
  // tile pair (j, j+1) trades the odd 16-lane rows (fq = 1, 3) of tile j against the even rows of
  // tile j+1, after which lane (fr, fq) holds the 8 contiguous channels 16 (j + (fq & 1)) + 8 (fq >> 1)
  // .. +7 of its pixel: half the store instructions for the same bytes (the tail of this epilogue is
  // store-issue bound with every CU's workgroup storing at once)
  static_assert(TN % 2 == 0, "tile pairs");
  const int sw = 12 * (fq & 1);  // 16 (fq & 1) + 8 (fq >> 1) - 4 fq
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; j += 2) {
      const auto r0 = __builtin_amdgcn_permlane16_swap(pk[j][i][0], pk[j + 1][i][0], false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(pk[j][i][1], pk[j + 1][i][1], false, false);
      if (!SQR_ABL(a, 2)) *(u32x4*)(out + opix[i] + 16 * j + sw) = u32x4{r0[0], r1[0], r0[1], r1[1]};
      if constexpr (BNB) {
        if (a.bn_act) {  // the activation, same layout
          const auto q0 = __builtin_amdgcn_permlane16_swap(ak[j][i][0], ak[j + 1][i][0], false, false);
          const auto q1 = __builtin_amdgcn_permlane16_swap(ak[j][i][1], ak[j + 1][i][1], false, false);
          *(u32x4*)((uint16_t*)a.bn_act + opix[i] + 16 * j + sw) = u32x4{q0[0], q1[0], q0[1], q1[1]};
        }
      }
    }
  if (!BNB && a.stats)
    tile_stats<T, BN, WAVES_M, WAVES_N, TM, TN, NT>(pk, (float*)smem, wm, wn, fr, fq, tid,
                                                 a.stats + ((size_t)tile_m * 2) * a.Nout + n0,
                                                 a.stats + ((size_t)tile_m * 2 + 1) * a.Nout + n0,
                                                 tile_n == 0 ? a.stats + (size_t)a.ntm * 2 * a.Nout + tile_m : nullptr,
                                                 (float)BM);
#ifdef SQR_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  SQR_STAMP(4);
  SQR_STAMP_WRITE(a.tp);
  clock_end(a.tp);
}


// ============================================================================ layer-1 persistent
// Cin = Nout = 64, W = TW = 64 (ResNetSQ layer1 at 256x256 input; TH = 2-row tiles) or 128 (at
// 512x512 input, config 5; 1-row tiles), forward and backward-data.  One workgroup per band of
// consecutive TH-row tiles of one image (B = 64: a quarter image = 8 tiles at 64 x 64, 32 tiles at
// 128 x 128 per workgroup):
//  * each wave's share of the 3x3 weights (its 32 output channels x 576, 36 MFMA fragments) is
//    loaded once (through a coalesced LDS image in the prologue) and held in VGPRs;
//  * input rows live in an NSLOT-slot LDS ring (slot = (row + 1) % NSLOT; one image row + its 2 zero
//    halo columns per slot): a tile reads TH + 2 rows of which only TH are new; the new rows of tile
//    k+2 are loaded into registers during tile k's MFMA loop and written to the ring at the end of
//    tile k+1, so every input row is fetched once per band;
//  * the output tile is staged in LDS (in the prologue's weight-image region, free once the weights
//    are in registers) and written with 16-B coalesced stores during the next tile's MFMA loop;
//    BatchNorm partials accumulate in registers, one partial row per workgroup.
// A wave covers TH * TW / 2 consecutive pixels of the tile (2 x 2 waves: pixel half x channel half).
struct D3PArgs {
  const void* x;   // [N][H][TW][64]
  const void* w;   // [64][9][64]
  void* out;       // [N][H][TW][64]
  const void* addend;  // ACC launches: out = conv + addend (backward-data of a block input; may alias out)
  const uint8_t* addend_mask;  // nullable (ACC): the addend counts only where its bit is set
  const void* bn_x;        // BNB launches: the following BatchNorm's input x [N][H][TW][64] ...
  const uint8_t* bn_mask;  // ... its ReLU mask (1 bit / element) and ...
  const float* bn_mean;    // ... its batch mean: out = dgrad * mask, stats = its backward sums
  float* stats;    // nullable: BatchNorm partials [gridDim.x][2][64]
  const float* in_coef;  // BNIN launches: x is the PRE-activation of the preceding BatchNorm + ReLU,
  void* in_act;          // [2][64] its (scale, shift): the conv reads relu(x * scale + shift) and writes
  uint8_t* in_mask;      // that activation (in_act) and its ReLU mask (1 bit / element) as side outputs
                         // (both null: no side outputs, y and the statistics only)
  int H, bpi, tpb, flip;  // bands per image, 2-row tiles per band
  uint32_t xbytes, wbytes;
  unsigned long long* tp;  // nullable: clock probe slots
};

// STATS: the forward's BatchNorm partials (a.stats != NULL); the backward-data launches skip the
// per-tile accumulation entirely (it cost ~0.15 us per tile).
// ACC (backward-data): out = conv + addend.  The addend of tile k is loaded into registers at the
// start of iteration k (16-B pieces in the staged-store layout) and added when tile k is stored
// at the start of iteration k+1, so its latency hides behind a whole tile of MFMA work (the row
// loads issued in between are younger, so the compiler's vmcnt wait for the addend skips them).
// BNB (backward-data feeding a BatchNorm+ReLU backward: a BasicBlock's conv2 dgrad into bn1): the
// stored value is g = dgrad * [relu mask] and a.stats receives, per workgroup, the BatchNorm
// backward sums (sum g, sum g*(x - mean)) — what sqr_bn_bwd's separate reduction pass would read
// back.  x and the mask of tile k are prefetched like ACC's addend.
// BNIN (forward with STATS): BatchNorm apply + ReLU on load.  Every input row piece is transformed in
// registers before it enters the LDS ring -- the new rows of tile k+1 during tile k's MFMA loop, the
// first tile's rows in the prologue -- except the zero padding (rows / columns outside the image stay
// zero: the conv pads the activation, not its input), and the rows this band owns (not its halo rows)
// are written out as the activation and its mask, bitwise what sqr_bn's apply pass writes.
template <typename T, bool STATS, bool ACC = false, bool BNB = false, int TW = 64, int TH = 2, bool BNIN = false>
__global__ void __launch_bounds__(256) conv3p_kernel(D3PArgs a) {
  constexpr int C = 64, BN = 64, NW = 4, NT = 256, ROWB = 128;
  // 2 x 2 waves, each WM pixels x 32 channels = TM 32x32 MFMA accumulators
  // (v_mfma_f32_32x32x16_bf16: half the MFMA instructions of 16x16x32 for the same work, which
  // leaves the single wave per SIMD issue slots for its LDS reads)
  constexpr int WAVES_M = 2, WAVES_N = 2, WM = TH * TW / WAVES_M, WN = 32, TM = WM / 32;
  constexpr int SLOTR = (TW + 2 + 7) / 8 * 8;  // LDS rows per ring slot: TW pixels + 2 halo, whole pieces
  constexpr int PPR = SLOTR / 8;               // LDS-DMA pieces (8 rows = 1 KiB) per image row
  constexpr int NSLOT = TH + 2 <= 4 ? 4 : 8;   // the tile's TH + 2 rows; the next tile's new rows
                                               // replace its first TH
  constexpr int RING = NSLOT * SLOTR * ROWB;   // 36 KiB (TW 64) / 68 KiB (TW 128)
  constexpr int WB = 9 * BN * ROWB;            // 72 KiB: prologue weight image, LDS row (tap, n)
  constexpr int WPW = 9 * BN / (8 * NW);       // 18 weight pieces per wave
  constexpr int STG = TH * TW * BN * 2;        // 16 KiB staged output tile (in the weight image's region)
  constexpr int NST = STG / 16 / NT;           // 16-B stores per thread per tile
  static_assert(TW % 32 == 0 && TM * 32 == WM && WN == 32, "a wave's pixels are whole 32-pixel runs of rows");
  static_assert(STG <= WB, "the staged tile fits the weight image's region");
  static_assert(2 * WAVES_M * 32 * BN * 4 <= RING && NT * 16 * 4 <= RING, "statistics scratch fits the ring");
  static_assert(NST <= 8, "store schedule");
  static_assert(!BNIN || (STATS && !ACC && !BNB), "apply-on-load: forward launches only");
  __shared__ __attribute__((aligned(1024))) char smem[WB + RING];  // 108 / 140 KiB
  __shared__ __attribute__((aligned(16))) float bnc[BNIN ? 128 : 4];  // BNIN: scale[64], shift[64]
  char* const wl = smem + RING;
  char* const ring = smem;
  char* const stg = wl;
  clock_begin(a.tp);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int prow = lane >> 3, pslot = lane & 7;
  constexpr uint32_t kOOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t xsrd = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsrd = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, a.wbytes, 0x00020000);
  const int H = a.H, ntile = a.tpb;
  const int img = blockIdx.x / a.bpi;
  const int hb = (blockIdx.x - img * a.bpi) * ntile * TH;  // first output row of the band

  // All global -> LDS traffic is register-staged (buffer_load_dwordx4 into VGPRs, ds_write_b128
  // later): an LDS-DMA piece costs this single wave per SIMD 60-185 issue cycles (MI355X guide,
  // cycle constants; measured here: ~1,000 cycles per tile of row issue and a ~7,000-cycle
  // prologue with LDS-DMA, tools/conv_phase.py), a plain load + ds_write a few tens.  Every LDS
  // image is the one the DMA wrote: lane L of a 1-KiB piece holds LDS row base + L/8, 16-B slot
  // L%8, and the XOR swizzle is applied on the source side.
  // Input rows r0 .. r0+nrows-1 (row -1 / H: zero padding via the buffer range check); piece p
  // (8 LDS rows of one image row) belongs to wave p % 4.
  constexpr int RPW = (TH * PPR + NW - 1) / NW;  // row pieces per wave for a tile's TH new rows (5)
  constexpr int PRW = ((TH + 2) * PPR + NW - 1) / NW;  // ... for the TH + 2 rows of the first tile
  // (use = false: every lane's offset is out of range -- no memory access, and the instruction count
  // stays the same on every path, so the compiler's vmcnt waits stay exact)
  auto row_piece = [&](int r0, int p, uint32_t* vo, bool use = true) {  // -> LDS byte offset of this lane's 16 B
    const int j = p / PPR, part = p - j * PPR;
    const int row = r0 + j;
    const int lbase = ((row + 1) & (NSLOT - 1)) * SLOTR + part * 8;  // first LDS row of the piece
    const int L = lbase + prow, w = part * 8 + prow - 1;
    const bool ok = use && (unsigned)row < (unsigned)H && (unsigned)w < (unsigned)TW;
    // the lane fetches channel group pslot and writes it to the swizzled slot pslot ^ key(L): the same
    // LDS image as a fetch of the swizzled group into slot pslot, but every piece a lane handles holds
    // the same 8 channels (BNIN keeps their coefficients in registers)
    *vo = ok ? (uint32_t)((((img * H + row) * TW + w) * C) * 2 + (pslot << 4)) : kOOB;
    return L * ROWB + ((pslot ^ ((L >> 1) & 7)) << 4);
  };
  auto load_rows = [&](int r0, int nrows, u32x4* v, bool use) {  // every wave issues the same count
#pragma unroll
    for (int i = 0; i < PRW; ++i) {
      const int p = i * NW + wave;
      if (i < (nrows * PPR + NW - 1) / NW) {  // compile-time
        uint32_t vo;
        row_piece(r0, p, &vo, use && p < nrows * PPR);
        v[i] = __builtin_amdgcn_raw_buffer_load_b128(xsrd, vo, 0, 0);
      }
    }
  };
  auto load_row_piece = [&](int r0, int i, u32x4* v, bool use) {  // piece i of TH rows (RPW per wave)
    const int p = i * NW + wave;
    uint32_t vo;
    row_piece(r0, p, &vo, use && p < TH * PPR);
    v[i] = __builtin_amdgcn_raw_buffer_load_b128(xsrd, vo, 0, 0);
  };
  auto write_rows = [&](int r0, int nrows, const u32x4* v) {
#pragma unroll
    for (int i = 0; i < PRW; ++i) {
      const int p = i * NW + wave;
      if (i * NW + NW <= nrows * PPR || p < nrows * PPR) {
        uint32_t vo;
        *(u32x4*)(ring + row_piece(r0, p, &vo)) = v[i];
      }
    }
  };

  float isc[BNIN ? 8 : 1], ish[BNIN ? 8 : 1];  // BNIN: (scale, shift) of channels 8 pslot .. +7
  // BNIN: piece p of the nrows rows from r0 (the lane's 16 B of it, as row_piece maps them) ->
  // relu(v * scale + shift) in place; the band's own rows also go out as the activation + mask
  auto bn_in_piece = [&](int r0, int nrows, int p, u32x4& v) {
    if constexpr (BNIN) {
      const int j = p / PPR, part = p - j * PPR;
      const int row = r0 + j;
      const int w = part * 8 + prow - 1;
      if (p < nrows * PPR && (unsigned)row < (unsigned)H && (unsigned)w < (unsigned)TW) {
        const int cg = pslot;  // the 8 channels every piece of this lane holds (row_piece)
        uint32_t mb = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float o0 = fmaxf(fmaf(lo2f<T>(v[e]), isc[2 * e], ish[2 * e]), 0.f);
          const float o1 = fmaxf(fmaf(hi2f<T>(v[e]), isc[2 * e + 1], ish[2 * e + 1]), 0.f);
          v[e] = pack2<T>(o0, o1);
          mb |= (lo2f<T>(v[e]) > 0.f ? 1u : 0u) << (2 * e);
          mb |= (hi2f<T>(v[e]) > 0.f ? 1u : 0u) << (2 * e + 1);
        }
        if (a.in_act && row >= hb && row < hb + TH * ntile) {
          const size_t pix = ((size_t)img * H + row) * TW + w;
          *(u32x4*)((char*)a.in_act + pix * C * 2 + cg * 16) = v;
          a.in_mask[pix * 8 + cg] = (uint8_t)mb;
        }
      }
    }
  };

  // 32x32x16 operand lanes: row r32 = lane & 31 (pixel / output channel), k half h = lane >> 5
  const int flip = a.flip;
  // BatchNorm statistics (this lane: pixel column, 16 channels wn*32 + 8g + 4h + e) over all tiles:
  // sums of the values shifted by K = the channel's first value in pixel lane r32 = 0 (broadcast at
  // tile 0, shared by the wave's 32 pixel lanes of that channel, so their sums add exactly in the
  // final xor tree; no cancellation while the values stay within a few std of K)
  // STATS: this thread's 8 channels (slot tid & 7: every staged piece it stores holds them) summed
  // over the pixels of its pieces as values shifted by the first one it stores (k, sum d, sum d^2),
  // accumulated while the piece goes out -- inside the next tile's MFMA loop, not after it
  float sk[STATS ? 8 : 1], ss[STATS ? 8 : 1], sq[STATS ? 8 : 1];
#pragma unroll
  for (int e = 0; e < (STATS ? 8 : 1); ++e) sk[e] = ss[e] = sq[e] = 0.f;

  u32x4 av[NST];  // ACC: the addend pieces of the tile stored next; BNB: the BatchNorm input x there
  uint32_t bm[(BNB || ACC) ? NST : 1];  // BNB / masked ACC: the mask byte of each piece (8 channels)
  float bs1[BNB ? 8 : 1], bs2[BNB ? 8 : 1], bmu[BNB ? 8 : 1];  // BNB: this thread's 8 channels (tid & 7)
  if constexpr (BNB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bs1[e] = bs2[e] = 0.f;
      bmu[e] = a.bn_mean[(tid & 7) * 8 + e];
    }
  }
  auto load_addend_piece = [&](int k, int q) {
    const size_t tile0 = ((size_t)img * H + hb + k * TH) * TW * BN;  // first element of tile k
    const char* src = (const char*)(BNB ? a.bn_x : a.addend) + tile0 * 2;
    av[q] = *(const u32x4*)(src + (size_t)(q * NT + tid) * 16);
    if constexpr (BNB) bm[q] = a.bn_mask[tile0 / 8 + q * NT + tid];
    if constexpr (ACC) bm[q] = a.addend_mask ? a.addend_mask[tile0 / 8 + q * NT + tid] : 0xffu;
  };
  // (use = false: a tile that does not exist -- the stores go out of the buffer's range and are
  // dropped; issuing them anyway keeps the vector-memory instruction count the same on every path,
  // so the compiler's vmcnt waits for the row registers never include these stores)
  const __amdgpu_buffer_rsrc_t osrd = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, a.xbytes, 0x00020000);
  auto store_piece = [&](int k, bool use, int q) {
    const uint32_t dst = use ? (uint32_t)(((img * H + hb + k * TH) * TW * BN) * 2) : kOOB;
    {
      const int c = q * NT + tid, row = c >> 3, slot = c & 7;
      u32x4 v = *(const u32x4*)(stg + row * ROWB + ((slot ^ ((row ^ (row >> 3)) & 7)) << 4));
      if constexpr (STATS) {
        if (use) {
          const bool first = k == 0 && q == 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = lo2f<T>(v[e]), hi = hi2f<T>(v[e]);
            if (first) {
              sk[2 * e] = lo;
              sk[2 * e + 1] = hi;
            }
            const float d0 = lo - sk[2 * e], d1 = hi - sk[2 * e + 1];
            ss[2 * e] += d0;
            sq[2 * e] = fmaf(d0, d0, sq[2 * e]);
            ss[2 * e + 1] += d1;
            sq[2 * e + 1] = fmaf(d1, d1, sq[2 * e + 1]);
          }
        }
      }
      if constexpr (ACC) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t ad = av[q][e] & ((((bm[q] >> (2 * e)) & 1u) ? 0xffffu : 0u) |
                                          (((bm[q] >> (2 * e + 1)) & 1u) ? 0xffff0000u : 0u));
          v[e] = pack2<T>(lo2f<T>(v[e]) + lo2f<T>(ad), hi2f<T>(v[e]) + hi2f<T>(ad));
        }
      }
      if constexpr (BNB) {
#pragma unroll
        for (int e = 0; e < 4 && use; ++e) {
          const uint32_t keep = (((bm[q] >> (2 * e)) & 1u) ? 0xffffu : 0u) | (((bm[q] >> (2 * e + 1)) & 1u) ? 0xffff0000u : 0u);
          v[e] &= keep;  // g = dgrad * mask (masked halves become +0)
          const float g0 = lo2f<T>(v[e]), g1 = hi2f<T>(v[e]);
          bs1[2 * e] += g0;
          bs2[2 * e] = fmaf(g0, lo2f<T>(av[q][e]) - bmu[2 * e], bs2[2 * e]);
          bs1[2 * e + 1] += g1;
          bs2[2 * e + 1] = fmaf(g1, hi2f<T>(av[q][e]) - bmu[2 * e + 1], bs2[2 * e + 1]);
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(v, osrd, dst | (uint32_t)(c * 16), 0, 0);
    }
  };
  auto store_staged = [&](int k, bool use) {
#pragma unroll
    for (int q = 0; q < NST; ++q) store_piece(k, use, q);
  };

  // Weights resident in REGISTERS: a wave's MFMA A operands for all 36 (tap, 16-channel slice)
  // steps (its 32 output channels x 576 = 36 KiB, 144 VGPRs; one wave per SIMD has 512), read once
  // from a coalesced LDS image.  The loop's LDS traffic is then only the input-row fragments (1
  // ds_read_b128 per MFMA instead of 1.5).  Slice kk of tap t = k-elements 16kk + 8h .. +7 for
  // lane half h.
  const int r32 = lane & 31, h = lane >> 5;
  V8<T> wreg[36];
  // rvb[t & 1]: the new rows of tile t, loaded during tile t-2's MFMA loop, written to the ring at the
  // end of tile t-1 (about 1.5 tiles of load latency hidden)
  u32x4 rvb[2][RPW];
  if constexpr (BNIN) {
    if (tid < 128) bnc[tid] = a.in_coef[tid];
  }
  {
    u32x4 t0[PRW], wv[WPW];
    load_rows(hb - 1, TH + 2, t0, true);  // tile 0: rows hb-1 .. hb+TH
#pragma unroll
    for (int i = 0; i < WPW; ++i) {  // weight image: LDS row r = tap * 64 + n  <-  w[n][tap][0..63]
      const int r = (i * NW + wave) * 8 + prow;
      const int tap = r / BN, n = r - tap * BN;
      wv[i] = __builtin_amdgcn_raw_buffer_load_b128(
          wsrd, (uint32_t)(((n * 9 + tap) * C) * 2 + ((pslot ^ ((r >> 1) & 7)) << 4)), 0, 0);
    }
    if constexpr (BNIN) {
      __syncthreads();  // the coefficients
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        isc[e] = bnc[8 * pslot + e];
        ish[e] = bnc[64 + 8 * pslot + e];
      }
#pragma unroll
      for (int i = 0; i < PRW; ++i)
        if (i * NW + NW <= (TH + 2) * PPR || i * NW + wave < (TH + 2) * PPR) bn_in_piece(hb - 1, TH + 2, i * NW + wave, t0[i]);
    }
    write_rows(hb - 1, TH + 2, t0);
#pragma unroll
    for (int i = 0; i < WPW; ++i) *(u32x4*)(wl + ((i * NW + wave) * 8) * ROWB + lane * 16) = wv[i];
  }
  // tile 1's new rows (written during tile 0).  Row loads are always the last vector-memory
  // instructions before the loop head, so the compiler's vmcnt waits for them are exact on both
  // paths into the loop (a younger store would make it wait for the store as well)
  load_rows(hb + TH + 1, TH, rvb[1], ntile > 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  {
    const int prow32 = (wn * WN + r32) * ROWB, pkey = ((wn * WN + r32) >> 1) & 7;
#pragma unroll
    for (int s = 0; s < 36; ++s)
      wreg[s] = *(const V8<T>*)(wl + (s >> 2) * BN * ROWB + prow32 + (((2 * (s & 3) + h) ^ pkey) << 4));
  }

  // One tile = 36 MFMA steps.  Its vector-memory work is spread over those steps instead of issued
  // in bursts at the tile boundary (every workgroup runs in lock-step with the others, so bursts
  // leave HBM idle during the MFMA loops and saturated in between: the kernel without its MFMA loop
  // takes 11-13 us, with it 23-27 us): the NST (4) staged stores of tile k-1 at steps 1 + 8q, the
  // row loads of tile k+2 at steps 3 + 7i, the addend / BatchNorm-input loads of tile k at 5 + 8q.
  constexpr int SSP = 32 / NST, RSP = 35 / RPW;
  auto tile = [&](int k, auto par) {
    constexpr int P = decltype(par)::value;  // k & 1 (static: selects the row buffers)
    f32x16 acc[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    // tap (r, c3) of tile pixel (y, x) reads input row hb+TH*k+y+r-1 = ring slot (hb+TH*k+y+r) % NSLOT,
    // LDS row x + c3 of it
    const int rbase = hb + TH * k;
    // 36 (tap, 16-channel slice) steps; slice kk of a 128-B row = 16-B slots 2kk + h
    auto load = [&](int s, V8<T>* qf) {
      const int t = s >> 2, kk = s & 3;
      const int r = t / 3, c3 = t % 3;
      const int rr = flip ? 2 - r : r, cc = flip ? 2 - c3 : c3;
      const int slot = 2 * kk + h;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m0 = wm * WM + 32 * i;  // the 32-pixel run's first tile pixel (wave-uniform)
        const int L = ((rbase + m0 / TW + rr) & (NSLOT - 1)) * SLOTR + cc + (m0 % TW) + r32;
        qf[i] = *(const V8<T>*)(ring + L * ROWB + ((slot ^ ((L >> 1) & 7)) << 4));
      }
    };
    constexpr int NSTEP = 36, PD = 2;
    V8<T> qf[PD + 1][TM];
#pragma unroll
    for (int s = 0; s < PD; ++s) load(s, qf[s]);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      if (s % SSP == 1 && s / SSP < NST) store_piece(k - 1, k >= 1, s / SSP);
      if (s % RSP == 3 % RSP && s / RSP < RPW)
        load_row_piece(hb + TH * (k + 2) + 1, s / RSP, rvb[P], k + 2 < ntile);
      if constexpr (BNIN)  // tile k+1's new rows (loaded during tile k-1), before they enter the ring
        if (s % RSP == 5 % RSP && s / RSP < RPW && k + 1 < ntile)
          bn_in_piece(hb + TH * (k + 1) + 1, TH, (s / RSP) * NW + wave, rvb[1 - P][s / RSP]);
      if constexpr (ACC || BNB)
        if (s % SSP == 5 % SSP && s / SSP < NST) load_addend_piece(k, s / SSP);
      if (s + PD < NSTEP) load(s + PD, qf[(s + PD) % (PD + 1)]);
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i] = mfma32(wreg[s], qf[s % (PD + 1)][i], acc[i]);
#pragma unroll
      for (int g = 0; g < TM; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // a fragment read
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // its address VALU
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // an MFMA
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // lane holds D[n = wn*32 + 8g + 4h + e][pixel wm*64 + 32i + r32], g = reg >> 2, e = reg & 3
    uint32_t pk[TM][4][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        pk[i][g][0] = pack2<T>(acc[i][4 * g], acc[i][4 * g + 1]);
        pk[i][g][1] = pack2<T>(acc[i][4 * g + 2], acc[i][4 * g + 3]);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // all waves are done with tile k's rows and the staging area
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = wm * WM + 32 * i + r32;
      const int key = (m ^ (m >> 3)) & 7;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = wn * WN + 8 * g + 4 * h;
        *(u32x2*)(stg + m * ROWB + ((((n >> 3) ^ key) << 4) | ((n & 7) << 1))) = u32x2{pk[i][g][0], pk[i][g][1]};
      }
    }
    // tile k+1's new rows (loaded during tile k-1) into the slots of tile k's first TH rows
    if (k + 1 < ntile) write_rows(hb + TH * (k + 1) + 1, TH, rvb[1 - P]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // staged tile and tile k+1's rows visible
  };
  for (int k = 0; k < ntile; k += 2) {
    tile(k, std::integral_constant<int, 0>{});
    if (k + 1 < ntile) tile(k + 1, std::integral_constant<int, 1>{});
  }
  if (ntile > 0) store_staged(ntile - 1, true);
  // the per-workgroup statistics reductions below reuse the ring: every wave is past its last ring
  // read (the loop's final barriers).  All loads of a column are issued at once (full unroll) and
  // summed into 8 interleaved partials, combined in a fixed tree (deterministic): a serial chain of
  // LDS round trips here cost ~3,500 cycles per workgroup (tools/conv_phase.py)
  auto col_sum = [&](const float* src, int n, int stride) {
    float p8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 64; ++r)
      if (r < n) p8[r & 7] += src[r * stride];
    return ((p8[0] + p8[1]) + (p8[2] + p8[3])) + ((p8[4] + p8[5]) + (p8[6] + p8[7]));
  };
  if constexpr (BNB) {  // red[256 threads][16] -> per channel, the 32 threads of its slot
    float* red = (float*)ring;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[tid * 16 + e] = bs1[e];
      red[tid * 16 + 8 + e] = bs2[e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (tid < 2 * BN) {
      const int q = tid / BN, col = tid - q * BN, sl = col >> 3, e = col & 7;
      a.stats[((size_t)blockIdx.x * 2 + q) * BN + col] = col_sum(red + sl * 16 + 8 * q + e, NT / 8, 8 * 16);
    }
  }
  if constexpr (STATS) {  // per thread (mean, M2) of its 8 channels -> red[256][16] -> the 32 rows of a slot
    float* red = (float*)ring;
    const float n = (float)(NST * ntile);  // values per thread and channel
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sn = ss[e] / n;
      red[tid * 16 + e] = sk[e] + sn;
      red[tid * 16 + 8 + e] = fmaxf(sq[e] - ss[e] * sn, 0.f);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (tid < BN) {  // channel tid = slot sl, element e: rows tid' = sl + 8 r (fixed order)
      const int sl = tid >> 3, e = tid & 7;
      float mean, m2;
      lane_rows_merge(red + sl * 16 + e, red + sl * 16 + 8 + e, NT / 8, 8 * 16, n, &mean, &m2);
      a.stats[((size_t)blockIdx.x * 2) * BN + tid] = mean;
      a.stats[((size_t)blockIdx.x * 2 + 1) * BN + tid] = m2;
      if (tid == 0) a.stats[(size_t)gridDim.x * 2 * BN + blockIdx.x] = (float)(TH * TW * ntile);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  clock_end(a.tp);
}

// ============================================================================ stride-2 dgrad
// Backward-data of a 3x3 / stride-2 / pad-1 conv (ResNetSQ's first conv of layers 2-3) as ONE
// direct kernel.  dX pixel (2i+ph, 2j+pw) only receives the taps of its parity class:
//   class (ph, pw) has taps t < Rc, u < Sc (Rc = 1 + ph, Sc = 1 + pw) reading dY[i + ph - t][j + pw - u]
// (sqr_conv2d_bwd_data's classes; weights packed per class [C][Rc][Sc][K]).  A workgroup owns a
// TH x TW block of dY positions of one image and BN output channels; the dY halo window
// ((TH+1) x (TW+1) positions) of EVERY 64-channel chunk is staged once (all chunks resident), then
// the four classes run one after the other — each a shifted-window GEMM over its 1/2/2/4 taps with
// its own accumulators and epilogue — while the class/chunk/tap weight tiles stream through an
// LDS-DMA ring.  Replaces the implicit GEMM whose per-class K (128-512) was too short to amortise
// its pipeline (layer 2: 38 us at 0.25 of peak).
struct D3S2Args {
  const void* dy;  // [N][Ho][Wo][K]
  const void* w;   // parity classes back to back, class cl = [C][Rc][Sc][K]
  void* dx;        // [N][2Ho][2Wo][C]
  const void* addend;  // nullable: dx = dgrad + addend (may alias dx)
  int addend_s2;       // 1: the addend is compact [N][Ho][Wo][C], added to the (even, even) pixels only
  int N, Ho, Wo, K, C;
  int tiles_x, tiles_per_img, ntn;
  int cls_off[4];  // elements
  uint32_t dybytes, wbytes;
  unsigned long long* tp;  // nullable: clock probe slots
};

__host__ __device__ constexpr int s2_ntaps(int cl) { return (1 + (cl >> 1)) * (1 + (cl & 1)); }

template <typename T, int TH, int TW, int BN, int WAVES_M, int WAVES_N, int NCH, int PD>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N) conv3s2_dgrad_kernel(D3S2Args a) {
  constexpr int NW = WAVES_M * WAVES_N, ROWB = 128, STAGES = PD + 1;
  constexpr int BM = TH * TW, WM = BM / WAVES_M, WN = BN / WAVES_N, TM = WM / 16, TN = WN / 16;
  constexpr int WWID = TW + 1, WR = (TH + 1) * WWID;
  constexpr int WROWS = (WR + 8 * NW - 1) / (8 * NW) * (8 * NW);
  constexpr int WP = WROWS / (8 * NW), PB = BN / (8 * NW);
  constexpr int WIN = WROWS * ROWB, TILE_B = BN * ROWB;
  constexpr int NSTEP = 9 * NCH;
  static_assert(PB >= 1 && PB * 8 * NW == BN, "BN must be a multiple of 8 * waves");
  static_assert(TM >= 1 && TN >= 1 && WM % 16 == 0, "wave tile");
  constexpr int NWIN = NCH < 2 ? 1 : 2;  // double-buffered dY windows (chunk cc in slot cc & 1)
  static_assert(PB * (PD - 1) + WP <= 63, "vmcnt range");
  static_assert(PD <= 8, "the next window must land within its chunk's 9 steps");
  __shared__ __attribute__((aligned(1024))) char smem[NWIN * WIN + STAGES * TILE_B];
  char* const bring = smem + NWIN * WIN;
  clock_begin(a.tp);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_m = bid / a.ntn, tile_n = bid - tile_m * a.ntn;
  const int img = tile_m / a.tiles_per_img, trem = tile_m - img * a.tiles_per_img;
  const int ty = trem / a.tiles_x, tx = trem - ty * a.tiles_x;
  const int i0 = ty * TH, j0 = tx * TW, n0 = tile_n * BN;
  constexpr uint32_t kOOB = 0x80000000u;
  const int prow = lane >> 3, pslot = lane & 7;
  const __amdgpu_buffer_rsrc_t dsrd = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, 0, a.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsrd = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, a.wbytes, 0x00020000);

  // dY window of a chunk: window row r = (y, x) -> dY position (i0 + y, j0 + x)
  uint32_t wvoff[WP];
  {
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int r = (i * NW + wave) * 8 + prow;
      const int y = r / WWID, x = r - y * WWID;
      const int h = i0 + y, w = j0 + x;
      const bool ok = r < WR && h < a.Ho && w < a.Wo;
      wvoff[i] = ok ? (uint32_t)((((img * a.Ho + h) * a.Wo + w) * a.K) * 2 + ((pslot ^ d3key(r)) << 4)) : kOOB;
    }
  }
  auto issue_win = [&](int cc) {
    dma_pieces<WP, NW>(dsrd, smem + (cc & 1) * WIN, wvoff, __builtin_amdgcn_readfirstlane(cc * 128), wave);
  };
  issue_win(0);
  // weight tile of step q = 9 cc + s: chunk cc, class cl, tap tt (s = class offset + tt) -> rows
  // c = n0 + row of class cl
  int wrow[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) wrow[i] = n0 + (i * NW + wave) * 8 + prow;
  auto issue_w = [&](int q) {
    q = q < NSTEP ? q : NSTEP - 1;  // dummy reloads past the end keep the per-wave counts uniform
    const int cc = q / 9, s = q - 9 * cc;
    const int cl = s < 1 ? 0 : (s < 3 ? 1 : (s < 5 ? 2 : 3));
    const int nt = s2_ntaps(cl), tt = s - (cl == 0 ? 0 : (cl == 1 ? 1 : (cl == 2 ? 3 : 5)));
    uint32_t vo[PB];
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int rr = (i * NW + wave) * 8 + prow;
      vo[i] = (uint32_t)(((size_t)a.cls_off[cl] + ((size_t)wrow[i] * nt + tt) * a.K + cc * 64) * 2 +
                         ((pslot ^ d3key(rr)) << 4));
    }
    dma_pieces<PB, NW>(wsrd, bring + (q % STAGES) * TILE_B, vo, 0, wave);
  };
#pragma unroll
  for (int q = 0; q < PD; ++q) issue_w(q);
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PB * (PD - 1)) : "memory");
  __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fq = lane >> 4;
  int qbase[TM];  // window row of this lane's output position at offset (0, 0)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wm * WM + 16 * i + fr;
    qbase[i] = (m / TW) * WWID + (m % TW);
  }
  int poff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int row = wn * WN + 16 * j + fr;
    poff[j] = row * ROWB + ((fq ^ d3key(row)) << 4);
  }
  // all four classes stay in registers to the end: a per-class epilogue would write every other
  // pixel (partial lines) and its stores would hold up the next class's vmcnt waits
  f32x4 acc[4][TN][TM];
#pragma unroll
  for (int cl = 0; cl < 4; ++cl)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[cl][j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  int q = 0;
  for (int cc = 0; cc < NCH; ++cc) {
    const char* win = smem + (cc & 1) * WIN;
    const bool next_win = cc + 1 < NCH;
#pragma unroll
    for (int cl = 0; cl < 4; ++cl) {
      const int ph = cl >> 1, pw = cl & 1, Sc = 1 + pw, nt = s2_ntaps(cl);
#pragma unroll
      for (int tt = 0; tt < nt; ++tt, ++q) {
        issue_w(q + PD);
        // chunk cc + 1's window into the slot chunk cc - 1 used (every wave is past it)
        if (cl == 0 && next_win) issue_win(cc + 1);
        const int t = tt / Sc, u = tt - t * Sc;
        const int toff = (ph - t) * WWID + (pw - u);
        const char* bst = bring + (q % STAGES) * TILE_B;
        int qoff[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = qbase[i] + toff;
          qoff[i] = row * ROWB + ((fq ^ d3key(row)) << 4);
        }
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          V8<T> pf[TN], qf[TM];
#pragma unroll
          for (int j = 0; j < TN; ++j) pf[j] = *(const V8<T>*)(bst + (poff[j] ^ (sub << 6)));
#pragma unroll
          for (int i = 0; i < TM; ++i) qf[i] = *(const V8<T>*)(win + (qoff[i] ^ (sub << 6)));
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              acc[cl][j][i] = mfma(pf[j], qf[i], acc[cl][j][i]);
            }
        }
        // weight tile q+1 landed (tiles q+2 .. q+PD stay in flight; so does the next window while
        // it is younger than tile q+1, i.e. for the first PD-1 steps of the chunk)
        const int s = q - 9 * cc;
        if (next_win && s <= PD - 2)
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PB * (PD - 1) + WP) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PB * (PD - 1)) : "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
  }
  // epilogue, one output-row parity at a time: classes (ph, 0) and (ph, 1) interleave into a
  // [TH][2TW][BN] staging tile in the (now dead) window LDS, copied out as full 16-B pieces of
  // contiguous pixel rows.  Staging slot key (p >> 1) & 7 spreads a class's stride-2 pixels.
  constexpr int SL = BN / 8, PX = 2 * TW, HALF = TH * PX * SL;
  static_assert(TH * PX * BN * 2 <= NWIN * WIN + STAGES * TILE_B, "staging tile fits the LDS");
  if (TH * PX * BN * 2 > NWIN * WIN) {  // staging overlaps the weight ring: its dummy tail loads first
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }
  static_assert(SL >= 8, "staging swizzle assumes at least 8 slots per pixel");
  const int H = 2 * a.Ho, W = 2 * a.Wo;
  T* out = (T*)a.dx;
  // copy-out: 16-B pieces of contiguous dX rows (+ the addend's pieces, AG at a time: the 8-wave
  // layer-2 kernel has no registers to spare).  A half's first addend group is requested before
  // its staging writes so that its latency overlaps them.
  constexpr int NIT = (HALF + 64 * NW - 1) / (64 * NW), AG = NIT < 4 ? NIT : 4;
  static_assert(NIT % AG == 0, "addend groups");
  auto piece = [&](int it, int ph, int& p, int& sl, size_t& go) {
    const int idx = tid + it * 64 * NW;
    p = idx / SL;
    sl = idx - p * SL;
    const int y = p / PX, x = p - y * PX;
    go = (((size_t)img * H + 2 * (i0 + y) + ph) * W + 2 * j0 + x) * a.C + n0 + 8 * sl;
    return idx < HALF && i0 + y < a.Ho && j0 + (x >> 1) < a.Wo;
  };
  auto load_group = [&](int it0, int ph, uint4* av) {
#pragma unroll
    for (int u = 0; u < AG; ++u) {
      int p, sl;
      size_t go;
      if (piece(it0 + u, ph, p, sl, go)) {
        if (a.addend_s2) {  // compact addend: the (even, even) pixels of the ph = 0 half only
          const int y = p / PX, x = p - y * PX;
          av[u] = (x & 1) ? uint4{0u, 0u, 0u, 0u}
                          : *(const uint4*)((const T*)a.addend +
                                            (((size_t)img * a.Ho + i0 + y) * a.Wo + j0 + (x >> 1)) * a.C + n0 +
                                                8 * sl);
        } else {
          av[u] = *(const uint4*)((const T*)a.addend + go);
        }
      }
    }
  };
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    const bool add = a.addend && !(a.addend_s2 && ph == 1);
    uint4 av[AG];
    if (add) load_group(0, ph, av);
    if (ph) __syncthreads();  // previous half copied out
#pragma unroll
    for (int pw = 0; pw < 2; ++pw)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = wm * WM + 16 * i + fr;
        const int p = (m / TW) * PX + 2 * (m % TW) + pw;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = wn * WN + 16 * j + 4 * fq;
          const int slot = (n >> 3) ^ ((p >> 1) & 7);
          store4((T*)(smem + p * (BN * 2) + slot * 16 + (n & 4) * 2), acc[2 * ph + pw][j][i]);
        }
      }
    __syncthreads();
#pragma unroll
    for (int it0 = 0; it0 < NIT; it0 += AG) {
      if (it0 && add) load_group(it0, ph, av);
#pragma unroll
      for (int u = 0; u < AG; ++u) {
        int p, sl;
        size_t go;
        if (!piece(it0 + u, ph, p, sl, go)) continue;
        uint4 v = *(const uint4*)(smem + p * (BN * 2) + ((sl ^ ((p >> 1) & 7)) << 4));
        if (add) {
          uint32_t* vv = (uint32_t*)&v;
          const uint32_t* aa = (const uint32_t*)&av[u];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            vv[e] = pack2<T>(lo2f<T>(vv[e]) + lo2f<T>(aa[e]), hi2f<T>(vv[e]) + hi2f<T>(aa[e]));
        }
        *(uint4*)(out + go) = v;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the dummy tail loads
  clock_end(a.tp);
}

// ============================================================================ weight gradient
// dW[k][tap][c] = sum_p dY[p][k] * X[p + shift(tap)][c] over the pixels of the split.  A
// workgroup owns a 64 (k) x 64 (c) x 9 (taps) output block and walks its split's pixel chunks
// (TH x TW rectangles of one image): per chunk it stages the dY rows and the (TH+2) x (TW+2) X halo
// window (both pixel-major, 128-B rows, 32-B-window XOR swizzle) and runs 9 shifted GEMMs whose
// MFMA fragments come from ds_read_b64_tr_b16 transposing reads.  Wave w owns channels
// c0+16w..+15 for all 4 k-tiles and 9 taps: per 32-pixel k-step 4 dY + 9 X fragments feed
// 36 MFMAs, and per chunk one window serves all 9 taps (the implicit-GEMM TN kernel re-gathers X
// per tap).  Output: fp32 split slabs in torch's KCRS layout, summed by wgrad_sum_kernel.
// 32-B-window XOR key of an LDS pixel row by its (y, x) position in the tile/window:
// the half-wave tr16 reads touch pixels (y, x..x+3) and (y, x+8..x+11) (TW >= 16) or
// (y, x..x+3) and (y+1, x..x+3) (TW = 8); with 128-B rows the row parity (= x parity, widths are
// even) splits the 256-B bank cycle and this key separates the rest.  Because it depends on x and
// on the parity of y only, a tap shift by r rows keeps it (r even) or flips its bit 1 (r odd).
__device__ __forceinline__ int psw(int y, int x) { return ((x >> 1) & 1) | ((((x >> 3) ^ y) & 1) << 1); }

template <int OFF>
__device__ __forceinline__ s16x4 ds_read_tr16_off(uint32_t addr) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}

// compile-time loop: f(std::integral_constant<int, I>{}) for I = B .. E-1
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt field");
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(m * PER) for m in 0..2 (m wave-uniform; PER pieces per chunk)
template <int PER>
__device__ __forceinline__ void wait_vm_chunks(int m) {
  if (m >= 2) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
  } else if (m == 1) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// wgrad read stream: LDS reads still allowed in flight when step j (of NS per chunk) starts, i.e.
// the reads issued after step j's X fragments — 2 per step plus 8 dY reads ahead of each sub's
// tap 0 — by the D-1 steps since; in the last chunk nothing is issued past its end
constexpr int wg_lgkm(int j, int D, int NS, bool last) {
  int n = 0;
  for (int k = j - D + 1; k <= j - 1; ++k) {
    if (last && k + D >= NS) continue;
    n += 2 + ((k + D) % 9 == 0 ? 8 : 0);
  }
  return n > 15 ? 15 : n;
}

struct D3WArgs {
  const void* x;   // [N][H][W][C]
  const void* dy;  // [N][Ho][Wo][K]
  float* slab;     // [splits][K][C][9] (KCRS)
  int N, H, W, C, K, Ho, Wo;
  int tiles_x, chunks_per_img, nchunks, cps;  // cps = chunks per split
  int ntc, ntiles;                              // C/64, (K/64)*(C/64)
  uint32_t xbytes, dybytes;
  unsigned long long* tp;  // clock probe (null unless armed)
};

// X window geometry of the weight-gradient kernel.  Stride 1: one (TH+2) x (TW+2) plane.  Stride
// 2: the (2TH+1) x (2TW+1) input window as four phase planes (a, b) = (input row, column parity
// relative to the window origin), plane (a, b) holding TH+1-a rows of width TW+2 (b = 0: TW+1
// columns + one unused, keeping the width even for the XOR key) or TW (b = 1).  Tap (r, s) of
// output pixel (py, px) reads plane (r & 1, s & 1) at (py + (r >> 1), px + (s >> 1)): consecutive
// output pixels are consecutive plane rows, so the stride-1 fragment reads carry over.
template <int S, int TW, int TH>
struct WgWin {
  static constexpr int PH(int a) { return S == 1 ? TH + 2 : TH + 1 - a; }
  static constexpr int PW(int b) { return S == 1 ? TW + 2 : (b ? TW : TW + 2); }
  static constexpr int PB(int a, int b) {  // first LDS row of plane (a, b)
    return S == 1 ? 0 : (a * 2 + b >= 1 ? PH(0) * PW(0) : 0) + (a * 2 + b >= 2 ? PH(0) * PW(1) : 0) +
                            (a * 2 + b >= 3 ? PH(1) * PW(0) : 0);
  }
  static constexpr int ROWS = S == 1 ? PH(0) * PW(0) : PB(1, 1) + PH(1) * PW(1);
  static constexpr int YO(int r) { return S == 1 ? r : r >> 1; }  // tap -> plane row / column offset
  static constexpr int PA(int r) { return S == 1 ? 0 : r & 1; }   // tap -> plane parity
};

template <typename T, int TW, int TH, int STAGES, int S>
__global__ void __launch_bounds__(256) conv3_wgrad_kernel(D3WArgs a) {
  constexpr int NW = 4, ROWB = 128;
  constexpr int BKP = TW * TH, SUBS = BKP / 32;      // pixels per chunk, 32-pixel k-steps
  using Win = WgWin<S, TW, TH>;
  constexpr int WR = Win::ROWS;
  constexpr int WROWS = (WR + 31) / 32 * 32;
  constexpr int DP = BKP / 32, XP = WROWS / 32;      // dY / window pieces per wave per chunk
  constexpr int PER = DP + XP;
  constexpr int TILE_D = BKP * ROWB, STAGE = TILE_D + WROWS * ROWB;
  static_assert(BKP % 64 == 0, "chunk = multiple of 64 pixels");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  clock_begin(a.tp);
  SQR_STAMP_DECL
  SQR_STAMP(0);
  const int split = bid / a.ntiles, tile = bid - split * a.ntiles;
  const int k0 = (tile / a.ntc) * 64, c0 = (tile % a.ntc) * 64;
  const int ch0 = split * a.cps;
  const int nloc = min(a.nchunks - ch0, a.cps);

  // ---- per-lane DMA constants
  constexpr uint32_t kOOB = 0x80000000u;
  const int prow = lane >> 3, pslot = lane & 7;
  uint32_t dvoff[DP];  // dY: chunk-relative byte offset (the chunk origin goes in soffset)
#pragma unroll
  for (int i = 0; i < DP; ++i) {
    const int r = (i * NW + wave) * 8 + prow;  // local pixel
    const int lch = 2 * ((pslot >> 1) ^ psw(r / TW, r % TW)) + (pslot & 1);
    dvoff[i] = (uint32_t)((((r / TW) * a.Wo + (r % TW)) * a.K + k0 + lch * 8) * 2);
  }
  // window LDS row r -> plane (pa, pb), plane position (y, x) -> input offset (iy, ix) from the
  // chunk's window origin (S*h0 - 1, S*w0 - 1)
  int xwy[XP], xwx[XP], xcol[XP];
#pragma unroll
  for (int i = 0; i < XP; ++i) {
    const int r = (i * NW + wave) * 8 + prow;
    int pa = 0, pb = 0;
    if (S == 2) {
      pa = r >= Win::PB(1, 0) ? 1 : 0;
      pb = r >= Win::PB(1, 1) || (r >= Win::PB(0, 1) && r < Win::PB(1, 0)) ? 1 : 0;
    }
    const int pbase = pa ? (pb ? Win::PB(1, 1) : Win::PB(1, 0)) : (pb ? Win::PB(0, 1) : Win::PB(0, 0));
    const int pw = pb ? Win::PW(1) : Win::PW(0);
    const int y = (r - pbase) / pw, x = (r - pbase) - y * pw;
    const int lch = 2 * ((pslot >> 1) ^ psw(y, x)) + (pslot & 1);
    // padding rows of the LDS window and the unused column of the b = 0 planes fail the bounds test
    const bool used = r < WR && (S == 1 || x < TW + 1 - pb);
    xwy[i] = used ? S * y + pa : -(1 << 20);
    xwx[i] = S * x + pb;
    xcol[i] = (c0 + lch * 8) * 2;
  }
  int xlin[XP];  // window piece offset from the chunk origin's X byte offset (may be negative)
#pragma unroll
  for (int i = 0; i < XP; ++i) xlin[i] = xwy[i] < 0 ? 0 : (xwy[i] * a.W + xwx[i]) * a.C * 2 + xcol[i];
  const __amdgpu_buffer_rsrc_t xsrd = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dsrd = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, 0, a.dybytes, 0x00020000);

  // ---- fragment addressing: lane (fq, fr) reads pixels kk = 32*sub + 8*fq + (fr>>2) (+4) at
  // byte 8*(fr&3) of the 32-B window holding its 16 columns (TN kernel convention)
  const int fr = lane & 15, fq = lane >> 4;
  // sub-0 offsets in two row-parity variants: sub s shifts the pixels by (32s/TW rows, 32s%TW
  // columns) and tap (r, s) the window by r rows more; a column shift of 32 keeps the XOR key and
  // an odd row shift flips its bit 1 (address bit 6), so every read is sbase + one of these
  // registers + an immediate offset
  int dpar[2][2][4];  // [row parity][h][k-tile] dY fragment offsets
  int xpar[2][2][3];  // [row parity][h][column tap] window fragment offsets (row tap 0)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kk = 8 * fq + (fr >> 2) + 4 * h;
    const int py = kk / TW, px = kk % TW;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      dpar[0][h][kt] = kk * ROWB + ((kt ^ psw(py, px)) << 5) + 8 * (fr & 3);
      dpar[1][h][kt] = dpar[0][h][kt] ^ 64;
    }
#pragma unroll
    for (int c3 = 0; c3 < 3; ++c3) {
      const int pb = Win::PA(c3), xo = Win::YO(c3);
      xpar[0][h][c3] = (Win::PB(0, pb) + py * Win::PW(pb) + px + xo) * ROWB + ((wave ^ psw(py, px + xo)) << 5) +
                       8 * (fr & 3);
      xpar[1][h][c3] = xpar[0][h][c3] ^ 64;
    }
  }

  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) acc[t][kt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // The chunk's 9*SUBS steps (sub, tap) run as one flat stream: a step's 4 MFMAs are followed by
  // the LDS reads of the step D later (its X fragments, and the dY fragments of a new sub), so a
  // read has D steps (D*64 MFMA cycles) to land before anything waits on it, and the stream
  // carries across chunk boundaries.  Two barriers per chunk: A at step 0 (every wave is past the
  // previous chunk's stage -> the DMA for chunk q+STAGES-1 may overwrite it) and T at step NS-D
  // (chunk q+1 has landed -> its reads may start).  The stage of a chunk is a compile-time
  // constant (the chunk loop is unrolled by STAGES) so that every read is one of the per-stage
  // base registers + an immediate: no address arithmetic in the stream (with one wave per SIMD
  // the instruction issue between the MFMAs is what the stream is short of).
  constexpr int NS = 9 * SUBS, D = 4;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x4 xlo[9], xhi[9], dlo[2][4], dhi[2][4];
  uint32_t dps[STAGES][2][2][4], xps[STAGES][2][2][3];
  {
    const uint32_t sm0 = lds_addr(smem);
#pragma unroll
    for (int st = 0; st < STAGES; ++st)
#pragma unroll
      for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) dps[st][par][h][kt] = sm0 + st * STAGE + dpar[par][h][kt];
#pragma unroll
          for (int c3 = 0; c3 < 3; ++c3) xps[st][par][h][c3] = sm0 + st * STAGE + TILE_D + xpar[par][h][c3];
        }
  }
  auto issue = [&](auto stc, auto jc) __attribute__((always_inline)) {
    constexpr int ST = decltype(stc)::value, jn = decltype(jc)::value;
    constexpr int s = jn / 9, t = jn % 9, R = t / 3, Sc = t % 3;
    constexpr int DYS = 32 * s / TW, DXS = 32 * s % TW;  // sub s's pixel shift
    if constexpr (t == 0) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        dlo[s & 1][kt] = ds_read_tr16_off<32 * s * ROWB>(dps[ST][DYS & 1][0][kt]);
        dhi[s & 1][kt] = ds_read_tr16_off<32 * s * ROWB>(dps[ST][DYS & 1][1][kt]);
      }
    }
    constexpr int PB_ = Win::PA(Sc), YR = DYS + Win::YO(R);
    constexpr int XOFF = (Win::PB(Win::PA(R), PB_) - Win::PB(0, PB_) + YR * Win::PW(PB_) + DXS) * ROWB;
    static_assert(XOFF < 65536, "ds offset field");
    xlo[t] = ds_read_tr16_off<XOFF>(xps[ST][YR & 1][0][Sc]);
    xhi[t] = ds_read_tr16_off<XOFF>(xps[ST][YR & 1][1][Sc]);
  };
  // chunk q in stage ST (= q % STAGES); LAST: no chunk follows
  // the chunk whose DMA is being issued: window origin (input coordinates), dY / X byte offsets
  int pl_oy = 0, pl_ox = 0, pl_dso = 0, pl_xo = 0;
  auto plan = [&](int ch) __attribute__((always_inline)) {
    const int img = ch / a.chunks_per_img, rem = ch - img * a.chunks_per_img;
    const int ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
    const int h0 = ty * TH, w0 = tx * TW;
    pl_oy = S * h0 - 1;
    pl_ox = S * w0 - 1;
    pl_dso = __builtin_amdgcn_readfirstlane(((img * a.Ho + h0) * a.Wo + w0) * a.K * 2);
    pl_xo = __builtin_amdgcn_readfirstlane(((img * a.H + pl_oy) * a.W + pl_ox) * a.C * 2);
  };
  // piece i of the planned chunk into stage st: dY pieces first, then the window's
  auto piece = [&](auto ic, int st) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    if constexpr (i < DP) {
      dma_piece(dsrd, smem + st * STAGE + ((i * NW + wave) * 8) * 128, dvoff[i], pl_dso);
    } else {
      constexpr int xi = i - DP;
      const int h = pl_oy + xwy[xi], w = pl_ox + xwx[xi];
      const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      const uint32_t vo = (uint32_t)(pl_xo + xlin[xi]) | (ok ? 0u : kOOB);
      dma_piece(xsrd, smem + st * STAGE + TILE_D + ((xi * NW + wave) * 8) * 128, vo, 0);
    }
  };
  auto chunk = [&](auto stc, auto lastc, int q) __attribute__((always_inline)) {
    constexpr int ST = decltype(stc)::value, NX = (ST + 1) % STAGES;
    constexpr bool LAST = decltype(lastc)::value;
    static_assert(PER < NS - D, "a chunk's DMA pieces are all issued before barrier T");
    const bool more = q + STAGES - 1 < nloc;
    static_for<0, NS>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      constexpr int s = j / 9, t = j % 9;
      lgkm_wait<wg_lgkm(j, D, NS, LAST)>();
      __builtin_amdgcn_sched_barrier(0);
      const s16x8 xv = {xlo[t][0], xlo[t][1], xlo[t][2], xlo[t][3], xhi[t][0], xhi[t][1], xhi[t][2], xhi[t][3]};
      const V8<T> afr = __builtin_bit_cast(V8<T>, xv);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const s16x4 &lo = dlo[s & 1][kt], &hi = dhi[s & 1][kt];
        const s16x8 dv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[t][kt] = mfma(afr, __builtin_bit_cast(V8<T>, dv), acc[t][kt]);
      }
      // the DMA of chunk q+STAGES-1 into the stage chunk q-1 used: planned at step 0 (after
      // barrier A), one 1-KiB piece per step after it so its address math spreads over the MFMAs
      if constexpr (j == 0) {
        __builtin_amdgcn_s_barrier();
        plan(ch0 + q + STAGES - 1);
      }
      if constexpr (j >= 1 && j <= PER) {
        constexpr int i = j - 1, DST = (ST + STAGES - 1) % STAGES;
        if (more) piece(std::integral_constant<int, i>{}, DST);
      }
      if constexpr (j + D < NS) {
        issue(stc, std::integral_constant<int, j + D>{});
      } else if constexpr (!LAST) {
        if constexpr (j + D == NS) {
          wait_vm_chunks<PER>(min(STAGES - 2, nloc - q - 2));
          __builtin_amdgcn_s_barrier();
        }
        issue(std::integral_constant<int, NX>{}, std::integral_constant<int, j + D - NS>{});
      }
    });
  };

  if (nloc > 0) {
#pragma unroll
    for (int q = 0; q < STAGES - 1; ++q)
      if (q < nloc) {
        plan(ch0 + q);
        static_for<0, PER>([&](auto ic) __attribute__((always_inline)) { piece(ic, q); });
      }
    wait_vm_chunks<PER>(min(STAGES - 2, nloc - 1));
    __builtin_amdgcn_s_barrier();
    SQR_STAMP(1);
    SQR_STAMP(2);  // (no chunk-0 stamp in this kernel: its chunks run as one unrolled stream)
    static_for<0, D>([&](auto jc) __attribute__((always_inline)) { issue(std::integral_constant<int, 0>{}, jc); });
    // groups of STAGES chunks with a successor, then the 1..STAGES remaining ones (the last of them
    // LAST) — straight-line bodies only: a branch between bodies inside the loop made the compiler
    // move the accumulators between AGPRs and VGPRs around every chunk
    int q = 0;
    for (; q + STAGES < nloc; q += STAGES)
      static_for<0, STAGES>([&](auto sc) __attribute__((always_inline)) { chunk(sc, std::false_type{}, q + decltype(sc)::value); });
    const int rem = nloc - q;
    static_for<1, STAGES + 1>([&](auto rc) __attribute__((always_inline)) {
      constexpr int RM = decltype(rc)::value;
      if (rem == RM) {
        static_for<0, RM - 1>([&](auto sc) __attribute__((always_inline)) { chunk(sc, std::false_type{}, q + decltype(sc)::value); });
        chunk(std::integral_constant<int, RM - 1>{}, std::true_type{}, q + RM - 1);
      }
    });
  }


  // ---- epilogue: the tile leaves in torch's KCRS order, slab[split][k][c][tap], so that the slabs
  // sum elementwise into the gradient (wgrad_sum_kernel: coalesced, no transpose).  Lane (fr, fq) of
  // wave w holds, for k = k0+16kt+fr, the 36 values (c = c0+16w+4fq+e, tap t): one contiguous 144-B
  // run of the KCRS row dw[k][c0..c0+63][0..8].  The runs are staged in LDS (KG k-tiles of 16 rows
  // per round; rows padded by 16 B so the 16 rows of a store start on different banks) and leave as
  // whole 2304-B rows in 16-B pieces.
  constexpr int RW = 64 * 9 + 4;  // staged row stride (floats)
  constexpr int KG = STAGES * STAGE >= 64 * RW * 4 ? 4 : 2;
  static_assert(STAGES * STAGE >= 16 * KG * RW * 4, "epilogue staging fits the pipeline's LDS");
  SQR_STAMP(3);
  __syncthreads();  // every wave is past its last fragment read of the pipeline stages
  float* __restrict__ stg = (float*)smem;
  float* __restrict__ slab = a.slab + ((size_t)split * a.K + k0) * a.C * 9 + (size_t)c0 * 9;
  const size_t krow = (size_t)a.C * 9;
  static_for<0, 4 / KG>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value * KG;
    if constexpr (g > 0) __syncthreads();  // the previous round's rows have left
#pragma unroll
    for (int kq = 0; kq < KG; ++kq) {
      float* dst = stg + (16 * kq + fr) * RW + (16 * wave + 4 * fq) * 9;
      static_for<0, 9>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        f32x4 v;
        v[0] = acc[(4 * j + 0) % 9][g + kq][(4 * j + 0) / 9];
        v[1] = acc[(4 * j + 1) % 9][g + kq][(4 * j + 1) / 9];
        v[2] = acc[(4 * j + 2) % 9][g + kq][(4 * j + 2) / 9];
        v[3] = acc[(4 * j + 3) % 9][g + kq][(4 * j + 3) / 9];
        *(f32x4*)(dst + 4 * j) = v;
      });
    }
    __syncthreads();
    for (int i = tid; i < 16 * KG * 144; i += 256) {
      const int r = i / 144, q = i - r * 144;
      // nontemporal: the slab is read once, by the sum launch (same-box A/B +0.15 %,
      // profiles/r05r_ab_wgrad_nontemporal_slab.txt)
      __builtin_nontemporal_store(*(const f32x4*)(stg + r * RW + 4 * q), (f32x4*)(slab + (size_t)(16 * g + r) * krow + 4 * q));
    }
  });
#ifdef SQR_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  SQR_STAMP(4);
  SQR_STAMP_WRITE(a.tp);
  clock_end(a.tp);
}

namespace {
struct D3Cfg {
  int id, BM, BN, threads, TW, TH, nwb, imgs;
};

int g_direct = 1;  // 0 off, 1 on when the grid is big enough, 2 whenever the shape fits
#ifdef SQR_EXPERIMENTS
// experiment builds: SQR_D3_CFG / SQR_S2F_CFG force a candidate id, SQR_EXP sets the ablation bits
int env_int(const char* n, int dflt) {
  const char* v = getenv(n);
  return v && *v ? atoi(v) : dflt;
}
#endif
int g_persist = 1;  // layer-1 persistent kernel (0: the tiled conv3_kernel; tests compare the two)
int g_deep_ring = 1;  // 1: the deep-weight-ring tiles (ids 7, 8, 10) first; 0: their 3-stage twins (1, 2, 5)


int pow2_log(int x) {
  int l = 0;
  while ((1 << l) < x) ++l;
  return (1 << l) == x ? l : -1;
}

// candidate configurations, in order of preference; the first that tiles the shape and gives
// enough workgroups wins
bool pick(int N, int H, int W, int Cin, int Nout, D3Cfg* out) {
  const int nch = Cin / 64;
  const D3Cfg cands[] = {
      // id BM   BN  thr  TW  TH nwb imgs
      {0, 256, 64, 256, 64, 4, 1, 1},    // Nout 64, Cin 64 (layer1; the persistent kernel takes W 64)
      // deeper weight rings first (bitwise the same results; B=64 fwd: layer2 24.8 vs 25.7 us,
      // layer3 23.5 vs 23.9, layer4 27.1 vs 28.4 -- scratch/d3_cfg.py)
      {7, 256, 128, 512, 32, 8, 2, 1},   // W 32 (layer2), 4-stage weight ring
      {8, 128, 128, 512, 16, 8, 2, 1},   // W 16 (layer3), 6-stage ring
      {10, 128, 64, 256, 8, 8, 2, 2},    // 8 x 8, two images per tile (layer4), 9-stage ring
      {1, 256, 128, 512, 32, 8, 2, 1},   // W 32, 3-stage ring
      {2, 128, 128, 512, 16, 8, 2, 1},   // W 16, 3-stage ring
      {5, 128, 64, 256, 8, 8, 2, 2},     // 8 x 8, two images per tile (half the weight traffic of id 3)
      {9, 128, 64, 256, 8, 8, 2, 2},     // id 5 with a 6-stage ring
      {3, 64, 128, 256, 8, 8, 2, 1},     // W 8 (layer4, odd batch)
      {4, 256, 64, 256, 16, 16, 2, 1},   // W 16, whole image per tile (slower than id 2 on layer3)
      {6, 256, 32, 256, 8, 8, 2, 4},     // 8 x 8, four images per tile
#ifdef SQR_EXPERIMENTS
      {20, 128, 64, 256, 16, 8, 2, 1},   // W 16 (layer3), 72 KiB: two workgroups per CU
      {21, 128, 64, 256, 32, 4, 2, 1},   // W 32 (layer2), 80 KiB: two workgroups per CU
#endif
  };
#ifdef SQR_EXPERIMENTS
  static const int force = env_int("SQR_D3_CFG", -1);
#else
  constexpr int force = -1;
#endif
  for (const D3Cfg& c : cands) {
    if (force >= 0 && c.id != force) continue;
    if (force < 0 && !g_deep_ring && (c.id == 7 || c.id == 8 || c.id == 10)) continue;
    if (c.id == 0 && !(Nout == 64 && nch == 1)) continue;
    if (c.id != 0 && Nout % c.BN) continue;
    if (W % c.TW || H % c.TH) continue;
    if (c.imgs > 1 && (c.TH != H || c.TW != W || N % c.imgs)) continue;
    if (c.nwb == 1 && nch != 1) continue;
    const long long tiles = (long long)(N / c.imgs) * (H / c.TH) * (W / c.TW) * (Nout / c.BN);
    if (tiles < 128 && g_direct < 2) continue;
    // measured (scratch/nt_tune.py, B=64): the direct kernel beats the implicit-GEMM one on every
    // ResNetSQ 3x3/s1 shape: layer2 25.0 vs 28.1 us, layer3 23.6 vs 29.7, layer4 29.1 vs 39.8
    *out = c;
    return true;
  }
  return false;
}
}  // namespace

namespace {
bool s2_pick(int Ho, int Wo, int K, int C, int* TH, int* TW, int* BN, int* nch) {
  if (K % 64 || C % 64) return false;
  *nch = K / 64;
  *BN = 64;
  // tile per channel geometry (the launches below are instantiated for these); any image size the
  // tile divides (256x256 input: layer 2 / 3 / 4 = 32 / 16 / 8 wide, 512x512: 64 / 32 / 16)
  if (C == 64 && K == 128) {  // layer 2
    *TH = 8; *TW = 32;
  } else if (C == 128 && K == 256) {  // layer 3
    *TH = 4; *TW = 16;
  } else if (C == 256 && K == 512) {  // layer 4
    *TH = 8; *TW = 8;
  } else {
    return false;
  }
  return Wo % *TW == 0 && Ho % *TH == 0;
}
}  // namespace

int conv3s2_dgrad_launch(int dtype, const void* dy, const void* w_cls, const int* cls_off, void* dx, int N, int Ho,
                         int Wo, int K, int C, hipStream_t st, const void* addend, int addend_s2) {
  if (g_direct == 0) return kNotHandled;
  int TH, TW, BN, nch;
  if (!s2_pick(Ho, Wo, K, C, &TH, &TW, &BN, &nch)) return kNotHandled;
  const size_t dybytes = (size_t)N * Ho * Wo * K * 2, wbytes = (size_t)9 * C * K * 2;
  if (dybytes >= (1u << 31) || (size_t)N * 4 * Ho * Wo * C * 2 >= (1u << 31)) return kNotHandled;
  D3S2Args a;
  a.dy = dy;
  a.w = w_cls;
  a.dx = dx;
  a.addend = addend;
  a.addend_s2 = addend && addend_s2 ? 1 : 0;
  a.N = N;
  a.Ho = Ho;
  a.Wo = Wo;
  a.K = K;
  a.C = C;
  a.tiles_x = Wo / TW;
  a.tiles_per_img = (Ho / TH) * a.tiles_x;
  a.ntn = C / BN;
  for (int i = 0; i < 4; ++i) a.cls_off[i] = cls_off[i];
  a.dybytes = (uint32_t)dybytes;
  a.wbytes = (uint32_t)wbytes;
  a.tp = probe_clock_take();
  // measured (N=64, rocprofv3): layer 2 17.9 us (8x32 tile, 5-deep weight ring, 8 waves), layer 3
  // 17.6 us (4x16 tile, two workgroups per CU), layer 4 20.0 us (one 8x8 image per tile; the
  // implicit GEMM: 39.6 / 23.2 / 23.7 us); 4x32 / 8x16 / BN 128 / 2x2-wave / deeper-ring variants were
  // slower
  const dim3 grid(N * a.tiles_per_img * a.ntn);
  probe_begin(st);
#ifdef SQR_EXPERIMENTS
  static const int xpd = env_int("SQR_S2D_PD", 0);  // experiment builds: another weight-ring depth
  if (xpd == 2 || xpd == 3 || xpd == 5) {
    SQR_DISPATCH16(dtype, T, {
      if (nch == 2) {
        if (xpd == 2) hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 8, 32, 64, 4, 2, 2, 2>), grid, dim3(512), 0, st, a);
        else if (xpd == 3) hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 8, 32, 64, 4, 2, 2, 3>), grid, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 8, 32, 64, 4, 2, 2, 5>), grid, dim3(512), 0, st, a);
      } else if (nch == 8) {
        if (xpd == 2) hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 8, 8, 64, 2, 2, 8, 2>), grid, dim3(256), 0, st, a);
        else if (xpd == 3) hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 8, 8, 64, 2, 2, 8, 3>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 8, 8, 64, 2, 2, 8, 5>), grid, dim3(256), 0, st, a);
      } else {
        if (xpd == 2) hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 4, 16, 64, 2, 2, 4, 2>), grid, dim3(256), 0, st, a);
        else if (xpd == 3) hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 4, 16, 64, 2, 2, 4, 3>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 4, 16, 64, 2, 2, 4, 5>), grid, dim3(256), 0, st, a);
      }
    });
    probe_end(st);
    SQR_HIP_LAUNCH_CHECK("conv3s2_dgrad_kernel");
    return 0;
  }
#endif
  SQR_DISPATCH16(dtype, T, {
    if (nch == 2)
      hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 8, 32, 64, 4, 2, 2, 5>), grid, dim3(512), 0, st, a);
    else if (nch == 8)
      hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 8, 8, 64, 2, 2, 8, 3>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((conv3s2_dgrad_kernel<T, 4, 16, 64, 2, 2, 4, 3>), grid, dim3(256), 0, st, a);
  });
  probe_end(st);
  SQR_HIP_LAUNCH_CHECK("conv3s2_dgrad_kernel");
  return 0;
}


// kNotHandled = not applicable (caller falls back to the implicit-GEMM path), 0 = launched, else error
// stride-2 forward tiles (output TH x TW, one image per tile; the four-plane window and the 3-stage
// weight ring fit 160 KiB): layer 2 (Cin 64: one window), layers 3-4 (Cin 128 / 256: two windows)
namespace {
struct D3S2FCfg {
  int id, BM, BN, threads, TW, TH, nwb;
};
bool pick_s2f(int N, int Ho, int Wo, int Cin, int Nout, D3S2FCfg* out) {
  const int nch = Cin / 64;
  const D3S2FCfg cands[] = {
      // id BM   BN  thr  TW  TH nwb
      {0, 128, 128, 512, 32, 4, 1},  // Cin 64, Wo 32 (layer 2; 512x512: Wo 64)
      {1, 64, 128, 256, 16, 4, 2},   // Wo 16 (layer 3; 512x512: layer 3 at Wo 32)
      {2, 64, 128, 256, 8, 8, 2},    // Wo 8 (layer 4; 512x512: Wo 16)
#ifdef SQR_EXPERIMENTS
      {10, 128, 128, 512, 32, 4, 1},  // id 0 with a 5-stage weight ring (160 KiB)
      {11, 64, 128, 256, 16, 4, 2},   // id 1, 5-stage ring
      {12, 64, 128, 256, 8, 8, 2},    // id 2, 5-stage ring
      {13, 64, 64, 256, 32, 2, 1},    // Cin 64: 2 x 32 output tiles, 68 KiB (two workgroups per CU)
      {14, 64, 64, 256, 16, 4, 1},    // Cin 64: 4 x 16 output tiles, 64 KiB (two workgroups per CU)
#endif
  };
#ifdef SQR_EXPERIMENTS
  static const int force = env_int("SQR_S2F_CFG", -1);
#else
  constexpr int force = -1;
#endif
  for (const D3S2FCfg& c : cands) {
    if (force >= 0 && c.id != force) continue;
    if ((c.nwb == 1) != (nch == 1)) continue;
    if (Nout % c.BN || Wo % c.TW || Ho % c.TH) continue;
    if ((long long)N * (Ho / c.TH) * (Wo / c.TW) * (Nout / c.BN) < 128 && g_direct < 2) continue;
    *out = c;
    return true;
  }
  return false;
}
}  // namespace

// tiled configurations with an apply-on-load (BNIN) instantiation
bool bnin_tiled_id(int id) { return id == 7 || id == 8 || id == 10 || id == 1 || id == 2 || id == 5; }
constexpr int kBninMaxC = 512;  // conv3_kernel's BNIN coefficient table

// Where the no-side-output path is also the faster one (config-2 step tables, profiles/r06e_c2_steps.txt
// against r06a_c2_steps.txt, per BasicBlock): the tiled 32- and 16-wide tiles (ids 7, 8) save the
// apply pass for +1.2 / +1.3 us on the forward (layers 2 and 3: -4 / -5 us per block).  Not the
// persistent layer-1 kernel (its side outputs cost the forward +12 us, the activation store the
// backward-data +9.4 us) nor the two-image 8x8 tiles (id 10: the window transform and the loss of the
// k20 key cost +7.4 us, more than layer 4's small apply pass).
int conv3_bnin_nso_ok(int N, int H, int W, int C, int K) {
  if (g_direct == 0 || C % 64 || K % 64 || pow2_log(W) < 0 || C > kBninMaxC) return 0;
  if (C == 64 && K == 64 && (W == 64 || W == 128) && H % (W == 64 ? 2 : 1) == 0 && g_persist) return 0;
  D3Cfg f, b;
  // the forward (C -> K, BNIN) and the backward-data (K -> C, BNB with coefficients) both direct
  return pick(N, H, W, C, K, &f) && (f.id == 7 || f.id == 8 || f.id == 1 || f.id == 2) && pick(N, H, W, K, C, &b)
             ? 1
             : 0;
}

int conv3_launch(int dtype, const void* x, const void* w, void* out, int N, int H, int W, int Cin, int Nout, int flip,
                 float* stats, int* stats_rows, hipStream_t st, const void* addend, const BnbArgs* bnb, int stride,
                 const uint8_t* addend_mask, const BnInArgs* bnin) {
  if (addend_mask && (!addend || stride != 1)) return kNotHandled;
  const bool persist_shape = Cin == 64 && Nout == 64 && (W == 64 || W == 128) && H % (W == 64 ? 2 : 1) == 0 && g_persist;
  if (bnin) {  // apply-on-load: stride-1 forwards with statistics
    if (stride != 1 || flip || addend || bnb || !stats || (!bnin->act) != (!bnin->mask)) return kNotHandled;
    // with side outputs (activation + mask): the persistent layer-1 kernel only
    if (bnin->act && !persist_shape) return kNotHandled;
  }
  if (bnb && bnb->act && !bnb->coef) return kNotHandled;  // the activation output needs the coefficients
  // the mask from the coefficients: the tiled kernels only (layer-1 bn1 keeps the forward's side outputs)
  if (bnb && bnb->coef && persist_shape) return kNotHandled;
  if (g_direct == 0) return kNotHandled;
  if (stride == 2) {  // forward only (H, W: the input size)
    if (flip || addend || bnb || H % 2 || W % 2 || Cin % 64 || Nout % 64) return kNotHandled;
    const int Ho = H / 2, Wo = W / 2;
    D3S2FCfg c;
    if (!pick_s2f(N, Ho, Wo, Cin, Nout, &c)) return kNotHandled;
    const size_t xbytes = (size_t)N * H * W * Cin * 2, wbytes = (size_t)Nout * 9 * Cin * 2;
    if (xbytes >= (1u << 31) || wbytes >= (1u << 31) || (size_t)N * Ho * Wo * Nout * 2 >= (1u << 31)) return kNotHandled;
    D3Args a = {};
    a.x = x;
    a.w = w;
    a.out = out;
    a.stats = stats;
    a.N = N;
    a.H = Ho;
    a.W = Wo;
    a.iH = H;
    a.iW = W;
    a.Cin = Cin;
    a.Nout = Nout;
    a.tiles_x = Wo / c.TW;
    a.tiles_per_img = (Ho / c.TH) * a.tiles_x;
    a.ntm = N * a.tiles_per_img;
    a.ntn = Nout / c.BN;
    a.xbytes = (uint32_t)xbytes;
    a.wbytes = (uint32_t)wbytes;
    a.tp = probe_clock_take();
    if (stats_rows) *stats_rows = a.ntm;
#ifdef SQR_EXPERIMENTS
    a.exp = env_int("SQR_EXP", 0);
    if (a.exp & 1) a.stats = nullptr;
#endif
    const dim3 grid(a.ntm * a.ntn), blk(c.threads);
    probe_begin(st);
    SQR_DISPATCH16(dtype, T, {
      switch (c.id) {
        case 0: hipLaunchKernelGGL((conv3_kernel<T, 128, 128, 4, 2, 32, 4, 1, 1, 2, false, false, 2>), grid, blk, 0, st, a); break;
        case 1: hipLaunchKernelGGL((conv3_kernel<T, 64, 128, 2, 2, 16, 4, 2, 1, 2, false, false, 2>), grid, blk, 0, st, a); break;
#ifdef SQR_EXPERIMENTS
        case 10: hipLaunchKernelGGL((conv3_kernel<T, 128, 128, 4, 2, 32, 4, 1, 1, 4, false, false, 2>), grid, blk, 0, st, a); break;
        case 11: hipLaunchKernelGGL((conv3_kernel<T, 64, 128, 2, 2, 16, 4, 2, 1, 4, false, false, 2>), grid, blk, 0, st, a); break;
        case 12: hipLaunchKernelGGL((conv3_kernel<T, 64, 128, 2, 2, 8, 8, 2, 1, 4, false, false, 2>), grid, blk, 0, st, a); break;
        case 13: hipLaunchKernelGGL((conv3_kernel<T, 64, 64, 2, 2, 32, 2, 1, 1, 2, false, false, 2>), grid, blk, 0, st, a); break;
        case 14: hipLaunchKernelGGL((conv3_kernel<T, 64, 64, 2, 2, 16, 4, 1, 1, 2, false, false, 2>), grid, blk, 0, st, a); break;
#endif
        default: hipLaunchKernelGGL((conv3_kernel<T, 64, 128, 2, 2, 8, 8, 2, 1, 2, false, false, 2>), grid, blk, 0, st, a); break;
      }
    });
    probe_end(st);
    SQR_HIP_LAUNCH_CHECK("conv3_kernel");
    return 0;
  }
  if (Cin % 64 || Nout % 64 || pow2_log(W) < 0) return kNotHandled;
  const size_t xbytes = (size_t)N * H * W * Cin * 2, wbytes = (size_t)Nout * 9 * Cin * 2;
  if (xbytes >= (1u << 31) || wbytes >= (1u << 31) || (size_t)N * H * W * Nout * 2 >= (1u << 31)) return kNotHandled;
  // the persistent kernel: 64-wide maps in 2-row tiles, 128-wide maps (512x512 input) in 1-row tiles
  // (measured at B=64, 128 x 128, rocprof-free clock probe: fwd+stats 140 -> 101 us, dgrad 112 -> 91,
  // dgrad+addend 146 -> 116 against the tiled kernel; 64-wide maps in 4-row tiles were slower than
  // 2-row ones: fwd 31.5 vs 30.8 us, dgrad+addend 31.7 vs 29.0)
  const int pth = W == 64 ? 2 : 1;  // rows per tile
  if (Cin == 64 && Nout == 64 && (W == 64 || W == 128) && H % pth == 0 && g_persist) {
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess) dev = 0;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    }
    // bands: the largest divisor of the per-image tile count giving about one workgroup per CU
    const int tpi = H / pth;
    int bpi = 1;
    for (int d = 1; d <= tpi; ++d)
      if (tpi % d == 0 && (long long)N * d <= ncu) bpi = d;
    D3PArgs p;
    p.x = x;
    p.w = w;
    p.out = out;
    p.addend = addend;
    p.addend_mask = addend_mask;
    p.bn_x = bnb ? bnb->x : nullptr;
    p.bn_mask = bnb ? bnb->mask : nullptr;
    p.bn_mean = bnb ? bnb->mean : nullptr;
    p.stats = stats;
    p.in_coef = bnin ? bnin->coef : nullptr;
    p.in_act = bnin ? bnin->act : nullptr;
    p.in_mask = bnin ? bnin->mask : nullptr;
    p.H = H;
    p.bpi = bpi;
    p.tpb = tpi / bpi;
    p.flip = flip;
    p.xbytes = (uint32_t)xbytes;
    p.wbytes = (uint32_t)wbytes;
    p.tp = probe_clock_take();
    const int grid = N * bpi;
    if (stats_rows) *stats_rows = grid;  // one partial row per workgroup
    probe_begin(st);
#define SQR_D3P_LAUNCH(TW_, TH_)                                                                      \
  if (bnin)                                                                                          \
    hipLaunchKernelGGL((conv3p_kernel<T, true, false, false, TW_, TH_, true>), dim3(grid), dim3(256), 0, st, p); \
  else if (bnb)                                                                                      \
    hipLaunchKernelGGL((conv3p_kernel<T, false, false, true, TW_, TH_>), dim3(grid), dim3(256), 0, st, p); \
  else if (stats)                                                                                    \
    hipLaunchKernelGGL((conv3p_kernel<T, true, false, false, TW_, TH_>), dim3(grid), dim3(256), 0, st, p); \
  else if (addend)                                                                                   \
    hipLaunchKernelGGL((conv3p_kernel<T, false, true, false, TW_, TH_>), dim3(grid), dim3(256), 0, st, p); \
  else                                                                                               \
    hipLaunchKernelGGL((conv3p_kernel<T, false, false, false, TW_, TH_>), dim3(grid), dim3(256), 0, st, p);
    SQR_DISPATCH16(dtype, T, {
      if (W == 128) {
        SQR_D3P_LAUNCH(128, 1)
      } else {
        SQR_D3P_LAUNCH(64, 2)
      }
    });
#undef SQR_D3P_LAUNCH
    probe_end(st);
    SQR_HIP_LAUNCH_CHECK("conv3p_kernel");
    return 0;
  }
  D3Cfg c;
  if (!pick(N, H, W, Cin, Nout, &c)) return kNotHandled;
  if (bnin && (!bnin_tiled_id(c.id) || Cin > kBninMaxC)) return kNotHandled;
#ifdef SQR_EXPERIMENTS
#define SQR_D3_EXP_CASES(ACC_, BNB_)                                                                                 \
    case 20: hipLaunchKernelGGL((conv3_kernel<T, 128, 64, 2, 2, 16, 8, 2, 1, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;   \
    case 21: hipLaunchKernelGGL((conv3_kernel<T, 128, 64, 2, 2, 32, 4, 2, 1, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;
#else
#define SQR_D3_EXP_CASES(ACC_, BNB_)
#endif
  D3Args a;
  a.x = x;
  a.w = w;
  a.out = out;
  a.addend = addend;
  a.addend_mask = addend_mask;
  a.bn_x = bnb ? bnb->x : nullptr;
  a.bn_mask = bnb ? bnb->mask : nullptr;
  a.bn_mean = bnb ? bnb->mean : nullptr;
  a.bn_coef = bnb ? bnb->coef : nullptr;
  a.bn_act = bnb ? bnb->act : nullptr;
  a.in_coef = bnin ? bnin->coef : nullptr;
  a.stats = stats;
  a.N = N;
  a.H = H;
  a.W = W;
  a.iH = H;
  a.iW = W;
  a.Cin = Cin;
  a.Nout = Nout;
  a.tiles_x = W / c.TW;
  a.tiles_per_img = (H / c.TH) * a.tiles_x;
  a.ntm = N / c.imgs * a.tiles_per_img;
  a.ntn = Nout / c.BN;
  a.flip = flip;
  a.xbytes = (uint32_t)xbytes;
  a.wbytes = (uint32_t)wbytes;
  a.tp = probe_clock_take();
  if (stats_rows) *stats_rows = a.ntm;
#ifdef SQR_EXPERIMENTS
  a.exp = env_int("SQR_EXP", 0);
  if (a.exp & 1) a.stats = nullptr;
#endif
  const dim3 grid(a.ntm * a.ntn), blk(c.threads);
  probe_begin(st);
#define SQR_D3_CASES(ACC_, BNB_)                                                                                   \
  switch (c.id) {                                                                                                  \
    case 0: hipLaunchKernelGGL((conv3_kernel<T, 256, 64, 4, 1, 64, 4, 1, 1, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;    \
    case 1: hipLaunchKernelGGL((conv3_kernel<T, 256, 128, 4, 2, 32, 8, 2, 1, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;   \
    case 2: hipLaunchKernelGGL((conv3_kernel<T, 128, 128, 4, 2, 16, 8, 2, 1, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;   \
    case 3: hipLaunchKernelGGL((conv3_kernel<T, 64, 128, 2, 2, 8, 8, 2, 1, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;     \
    case 4: hipLaunchKernelGGL((conv3_kernel<T, 256, 64, 4, 1, 16, 16, 2, 1, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;   \
    case 5: hipLaunchKernelGGL((conv3_kernel<T, 128, 64, 2, 2, 8, 8, 2, 2, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;     \
    case 6: hipLaunchKernelGGL((conv3_kernel<T, 256, 32, 4, 1, 8, 8, 2, 4, 2, ACC_, BNB_>), grid, blk, 0, st, a); break;     \
    case 7: hipLaunchKernelGGL((conv3_kernel<T, 256, 128, 4, 2, 32, 8, 2, 1, 3, ACC_, BNB_>), grid, blk, 0, st, a); break;   \
    case 8: hipLaunchKernelGGL((conv3_kernel<T, 128, 128, 4, 2, 16, 8, 2, 1, 5, ACC_, BNB_>), grid, blk, 0, st, a); break;   \
    case 9: hipLaunchKernelGGL((conv3_kernel<T, 128, 64, 2, 2, 8, 8, 2, 2, 5, ACC_, BNB_>), grid, blk, 0, st, a); break;     \
    SQR_D3_EXP_CASES(ACC_, BNB_)                                                                                   \
    default: hipLaunchKernelGGL((conv3_kernel<T, 128, 64, 2, 2, 8, 8, 2, 2, 8, ACC_, BNB_>), grid, blk, 0, st, a); break;    \
  }
  SQR_DISPATCH16(dtype, T, {
    if (bnin) {
      // apply-on-load instantiations: the first-choice tiles of ResNetSQ's layers 2-4 at 256 / 512 input
      switch (c.id) {
        // (id 7's tile with the 3-stage ring: the 4-stage one fills the 160 KiB without the table)
        case 1:
        case 7: hipLaunchKernelGGL((conv3_kernel<T, 256, 128, 4, 2, 32, 8, 2, 1, 2, false, false, 1, true>), grid, blk, 0, st, a); break;
        case 2: hipLaunchKernelGGL((conv3_kernel<T, 128, 128, 4, 2, 16, 8, 2, 1, 2, false, false, 1, true>), grid, blk, 0, st, a); break;
        case 8: hipLaunchKernelGGL((conv3_kernel<T, 128, 128, 4, 2, 16, 8, 2, 1, 5, false, false, 1, true>), grid, blk, 0, st, a); break;
        case 5: hipLaunchKernelGGL((conv3_kernel<T, 128, 64, 2, 2, 8, 8, 2, 2, 2, false, false, 1, true>), grid, blk, 0, st, a); break;
        default: hipLaunchKernelGGL((conv3_kernel<T, 128, 64, 2, 2, 8, 8, 2, 2, 8, false, false, 1, true>), grid, blk, 0, st, a); break;
      }
    } else if (bnb) {
      SQR_D3_CASES(false, true)
    } else if (addend) {
      SQR_D3_CASES(true, false)
    } else {
      SQR_D3_CASES(false, false)
    }
  });
#undef SQR_D3_CASES
  probe_end(st);
  SQR_HIP_LAUNCH_CHECK("conv3_kernel");
  return 0;
}

// ---------------------------------------------------------------- weight-gradient launcher
namespace {
struct D3WPlan {
  int TW, TH, splits, cps, nchunks, chunks_per_img, tiles_x, ntiles, Ho, Wo;
};
bool plan_w(int N, int H, int W, int C, int K, int stride, D3WPlan* p) {
  if (g_direct == 0 || C % 64 || K % 64 || (stride != 1 && stride != 2)) return false;
  if (stride == 2 && (H % 2 || W % 2)) return false;
  const int Ho = H / stride, Wo = W / stride;
  if (Wo < 8 || pow2_log(Wo) < 0) return false;
  // stride 1: chunks of 128 pixels (64 for W = 8), a taller window amortising its halo rows;
  // stride 2: 64-pixel chunks (the four-plane window of a 128-pixel chunk would not fit 3 stages)
  int TW, TH;
  if (stride == 1) {
    TW = Wo >= 64 ? 64 : Wo;
    TH = TW == 8 ? 8 : 128 / TW;
  } else {
    TW = Wo >= 32 ? 32 : Wo;
    TH = 64 / TW;
  }
  if (Ho % TH) return false;
  if ((size_t)N * H * W * C * 2 >= (1u << 31) || (size_t)N * Ho * Wo * K * 2 >= (1u << 31)) return false;
  p->TW = TW;
  p->TH = TH;
  p->Ho = Ho;
  p->Wo = Wo;
  p->tiles_x = Wo / TW;
  p->chunks_per_img = (Ho / TH) * p->tiles_x;
  p->nchunks = N * p->chunks_per_img;
  p->ntiles = (K / 64) * (C / 64);
  int splits = (256 + p->ntiles - 1) / p->ntiles;  // one workgroup per CU
  splits = splits > p->nchunks ? p->nchunks : splits;
  p->cps = (p->nchunks + splits - 1) / splits;
  p->splits = (p->nchunks + p->cps - 1) / p->cps;
  return true;
}
}  // namespace

size_t conv3w_slab_bytes(int N, int H, int W, int C, int K, int stride) {
  D3WPlan p;
  if (!plan_w(N, H, W, C, K, stride, &p)) return 0;
  return (size_t)p.splits * K * 9 * C * sizeof(float);
}

int conv3w_launch(int dtype, const void* x, const void* dy, float* slab, size_t slab_bytes, int N, int H, int W, int C,
                  int K, int* splits, hipStream_t st, int stride) {
  D3WPlan p;
  if (!plan_w(N, H, W, C, K, stride, &p)) return kNotHandled;
  if ((size_t)p.splits * K * 9 * C * sizeof(float) > slab_bytes) return kNotHandled;
  D3WArgs a;
  a.x = x;
  a.dy = dy;
  a.slab = slab;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.K = K;
  a.Ho = p.Ho;
  a.Wo = p.Wo;
  a.tiles_x = p.tiles_x;
  a.chunks_per_img = p.chunks_per_img;
  a.nchunks = p.nchunks;
  a.cps = p.cps;
  a.ntc = C / 64;
  a.ntiles = p.ntiles;
  a.xbytes = (uint32_t)((size_t)N * H * W * C * 2);
  a.dybytes = (uint32_t)((size_t)N * p.Ho * p.Wo * K * 2);
  a.tp = probe_clock_take();
  *splits = p.splits;
  const dim3 grid(p.splits * p.ntiles), blk(256);
  probe_begin(st);
  SQR_DISPATCH16(dtype, T, {
    if (stride == 1) {
      switch (p.TW) {
        case 64: hipLaunchKernelGGL((conv3_wgrad_kernel<T, 64, 2, 3, 1>), grid, blk, 0, st, a); break;
        case 32: hipLaunchKernelGGL((conv3_wgrad_kernel<T, 32, 4, 3, 1>), grid, blk, 0, st, a); break;
        case 16: hipLaunchKernelGGL((conv3_wgrad_kernel<T, 16, 8, 3, 1>), grid, blk, 0, st, a); break;
        default: hipLaunchKernelGGL((conv3_wgrad_kernel<T, 8, 8, 4, 1>), grid, blk, 0, st, a); break;
      }
    } else {
      switch (p.TW) {
        case 32: hipLaunchKernelGGL((conv3_wgrad_kernel<T, 32, 2, 3, 2>), grid, blk, 0, st, a); break;
        case 16: hipLaunchKernelGGL((conv3_wgrad_kernel<T, 16, 4, 3, 2>), grid, blk, 0, st, a); break;
        default: hipLaunchKernelGGL((conv3_wgrad_kernel<T, 8, 8, 3, 2>), grid, blk, 0, st, a); break;
      }
    }
  });
  probe_end(st);
  SQR_HIP_LAUNCH_CHECK("conv3_wgrad_kernel");
  return 0;
}

}  // namespace conv
}  // namespace sqr

extern "C" int sqr_conv_set_deep_ring(int on) {
  const int old = sqr::conv::g_deep_ring;
  sqr::conv::g_deep_ring = on ? 1 : 0;
  return old;
}

extern "C" int sqr_conv_set_direct(int mode) {
  const int old = sqr::conv::g_direct;
  sqr::conv::g_direct = mode < 0 ? 0 : (mode > 2 ? 2 : mode);
  return old;
}
