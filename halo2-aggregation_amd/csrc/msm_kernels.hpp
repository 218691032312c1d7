// msm_kernels.hpp -- Pippenger MSM kernels for gfx950.
//
// Replaces halo2 `best_multiexp` / `multiexp_serial` ([3P], called from
// /root/reference/examples/simple-example.rs:606,620,638-640,702,722).  The
// reference is a CPU bucket method (unsigned c-bit windows, one bucket array
// per window per rayon chunk).  This is an MI355X re-design of the same math:
//
//   1. k_sort_hist  one lane per scalar: Montgomery -> canonical, signed
//                   digits for all W windows (halves the bucket count), LDS
//                   histogram of (window, coarse bin) per block.   [HBM]
//   2. k_scan_*     exclusive scan of the block histograms (block sums, then
//                   each block adds the sums before it).
//   3. k_sort_coarse / k_sort_fine: two-level LDS bucket sort -> per window,
//                   point indices grouped by bucket (sign in bit 31) and the
//                   bucket offsets.                                [HBM]
//   4. k_accumulate every lane walks an equal-length slice of the concatenated
//                   sorted list, summing consecutive same-bucket points with
//                   XYZZ mixed additions (load-balanced regardless of the
//                   bucket-size distribution).      [VALU-int bound, dominant]
//   5. k_bucket_seg_q folds each bucket's slice-boundary chain and forms the
//                   segment sums of L1 = 4 buckets: S_j = sum B, T_j = sum i*B.
//   6. k_bucket_bits per bucket set: G_b = sum_{j: bit b of j} S_j and
//                   partial sums of T_j via LDS tree reductions (parallel form
//                   of sum_j j*S_j), converted to the Rust R = 2^256 layout as
//                   host terms.
// The host (host_ec.hpp) then evaluates sum_w 2^{o_w} (sum T + L1 * sum_b 2^b
// G_b + K B_K) as one Horner over absolute bit positions.
#pragma once
#include "coop29.hpp"
#include "curve29.hpp"

namespace pm {

constexpr uint32_t kNegBit = 0x80000000u;

// ------------------------------------------------------------ vector loads
template <class F>
__device__ __forceinline__ Aff<F> load_aff(const uint32_t* __restrict__ p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1], c = q[2], d = q[3];
  Aff<F> r;
  r.x.l[0] = a.x; r.x.l[1] = a.y; r.x.l[2] = a.z; r.x.l[3] = a.w;
  r.x.l[4] = b.x; r.x.l[5] = b.y; r.x.l[6] = b.z; r.x.l[7] = b.w;
  r.y.l[0] = c.x; r.y.l[1] = c.y; r.y.l[2] = c.z; r.y.l[3] = c.w;
  r.y.l[4] = d.x; r.y.l[5] = d.y; r.y.l[6] = d.z; r.y.l[7] = d.w;
  return r;
}
template <class F>
__device__ __forceinline__ void store_fe4(uint4* q, const Fe<F>& a) {
  q[0] = make_uint4(a.l[0], a.l[1], a.l[2], a.l[3]);
  q[1] = make_uint4(a.l[4], a.l[5], a.l[6], a.l[7]);
}
template <class F>
__device__ __forceinline__ Fe<F> load_fe4(const uint4* q) {
  uint4 a = q[0], b = q[1];
  Fe<F> r;
  r.l[0] = a.x; r.l[1] = a.y; r.l[2] = a.z; r.l[3] = a.w;
  r.l[4] = b.x; r.l[5] = b.y; r.l[6] = b.z; r.l[7] = b.w;
  return r;
}
template <class F>
__device__ __forceinline__ void store_xyzz(Xyzz<F>* dst, const Xyzz<F>& p) {
  uint4* q = reinterpret_cast<uint4*>(dst);
  store_fe4<F>(q + 0, p.X);
  store_fe4<F>(q + 2, p.Y);
  store_fe4<F>(q + 4, p.ZZ);
  store_fe4<F>(q + 6, p.ZZZ);
}
template <class F>
__device__ __forceinline__ Xyzz<F> load_xyzz(const Xyzz<F>* src) {
  const uint4* q = reinterpret_cast<const uint4*>(src);
  Xyzz<F> p;
  p.X = load_fe4<F>(q + 0);
  p.Y = load_fe4<F>(q + 2);
  p.ZZ = load_fe4<F>(q + 4);
  p.ZZZ = load_fe4<F>(q + 6);
  return p;
}

// ------------------------------------------------------- 1. window geometry
// W windows split the 256-bit range evenly: window w has width
// c_w = 256/W + (w < 256%W) and bit offset o_w = w*(256/W) + min(w, 256%W),
// so no window is left with a handful of bits (which would make a few giant
// buckets).  Signed digits: d in [-2^(c_w-1)+1, 2^(c_w-1)], code = |d| |
// sign<<31, code 0 = skip.  The top window never produces a carry because
// scalars are < 2^255.
template <int W, int NBITS = 256>
struct WinGeom {
  static constexpr int base = NBITS / W;
  static constexpr int extra = NBITS % W;
  static constexpr __host__ __device__ int width(int w) { return base + (w < extra ? 1 : 0); }
  static constexpr __host__ __device__ int offset(int w) { return w * base + (w < extra ? w : extra); }
};

// ----------------------------------------------------------------- 2. scan
constexpr int kScanThreads = 256;
constexpr int kScanPerThread = 16;
constexpr int kScanChunk = kScanThreads * kScanPerThread;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// exclusive block scan; lds needs (blockDim/64 + 1) words
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, nw = blockDim.x >> 6;
  const uint32_t incl = wave_incl_scan(v);
  if (lane == 63) lds[wave] = incl;
  __syncthreads();
  if (tid == 0) {
    uint32_t s = 0;
    for (int w = 0; w < nw; w++) {
      uint32_t x = lds[w];
      lds[w] = s;
      s += x;
    }
    lds[nw] = s;
  }
  __syncthreads();
  const uint32_t r = incl - v + lds[wave];
  total = lds[nw];
  __syncthreads();
  return r;
}

// The block histograms are stored in tiles (k_sort_hist): rows of `nblk`
// block counters, R = kScanChunk / nblk rows per tile, and inside a tile
// block-major (counter (row, blk) at blk * Rt + row % R, Rt = the tile's
// rows), so each histogram block writes runs of Rt counters instead of one
// 4-B store per row (2^20: 8 us, 2^22: 24 us of strided stores before).  A
// scan block covers one tile (chunk = R nblk) and reads it in logical
// (row, blk) order; R = 1 (nblk > kScanChunk / 2) is the plain row-major
// layout with chunk = kScanChunk.
struct ScanTiles {
  uint32_t chunk;  // counters per scan block (one tile)
  uint32_t R;      // rows per tile (1: row-major)
  uint32_t nblk;   // counters per row
  uint32_t rows;   // histogram rows (the sentinel follows them)
};
__host__ __device__ inline ScanTiles scan_tiles(uint32_t rows, uint32_t nblk) {
  const uint32_t R = nblk <= (uint32_t)kScanChunk / 2 ? (uint32_t)kScanChunk / nblk : 1u;
  return ScanTiles{R > 1 ? R * nblk : (uint32_t)kScanChunk, R, nblk, rows};
}
// physical index of histogram counter (row, blk)
__device__ __forceinline__ size_t tile_index(const ScanTiles& t, uint32_t row, uint32_t blk) {
  if (t.R == 1) return (size_t)row * t.nblk + blk;
  const uint32_t tt = row / t.R, r = row - tt * t.R, Rt = min(t.R, t.rows - tt * t.R);
  return (size_t)tt * t.R * t.nblk + (size_t)blk * Rt + r;
}

static __global__ void __launch_bounds__(kScanThreads) k_scan_reduce(const uint32_t* __restrict__ in, uint32_t N,
                                                             ScanTiles tl, uint32_t* __restrict__ bsum) {
  __shared__ uint32_t lds[kScanThreads / 64 + 1];
  const size_t b0 = (size_t)blockIdx.x * tl.chunk;
  const uint32_t cnt = (uint32_t)min((size_t)tl.chunk, N - b0);
  uint32_t s = 0;
  for (uint32_t k = threadIdx.x; k < cnt; k += kScanThreads) s += in[b0 + k];  // a sum: order-free
  uint32_t total;
  block_excl_scan(s, lds, total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

static __global__ void __launch_bounds__(kScanThreads) k_scan_down(const uint32_t* __restrict__ in, uint32_t N,
                                                           ScanTiles tl, const uint32_t* __restrict__ bsum,
                                                           uint32_t* __restrict__ offsets,
                                                           uint32_t* __restrict__ cursor) {
  __shared__ uint32_t lds[kScanThreads / 64 + 1];
  __shared__ uint32_t tile[kScanChunk];
  const size_t b0 = (size_t)blockIdx.x * tl.chunk;
  const uint32_t cnt = (uint32_t)min((size_t)tl.chunk, N - b0);
  for (uint32_t k = threadIdx.x; k < cnt; k += kScanThreads) tile[k] = in[b0 + k];  // coalesced
  __syncthreads();
  // logical element j of this block (row-major (row, blk) order) lives at
  // tile position blk * Rt + row % R inside the tile; the sentinel after the
  // last row maps to itself
  const size_t tiled_end = (size_t)tl.rows * tl.nblk;
  uint32_t Rt = 1;
  if (tl.R > 1) Rt = min(tl.R, tl.rows - blockIdx.x * tl.R);
  const uint32_t base = threadIdx.x * kScanPerThread;
  uint32_t v[kScanPerThread];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPerThread; k++) {
    const uint32_t j = base + k;
    uint32_t p = j;
    if (tl.R > 1 && b0 + j < tiled_end) {
      const uint32_t r = j / tl.nblk;
      p = (j - r * tl.nblk) * Rt + r;
    }
    v[k] = j < cnt ? tile[p] : 0u;
    s += v[k];
  }
  // this block's offset = sum of the block sums before it (replaces a
  // single-block scan launch of bsum: nb is a few hundred at 2^20 - 2^23)
  uint32_t pre = 0;
  for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kScanThreads) pre += bsum[i];
  uint32_t total;
  block_excl_scan(pre, lds, total);
  const uint32_t bpre = total;
  uint32_t run = block_excl_scan(s, lds, total) + bpre;
#pragma unroll
  for (int k = 0; k < kScanPerThread; k++) {
    if (base + k < cnt) {
      offsets[b0 + base + k] = run;
      if (cursor) cursor[b0 + base + k] = run;
    }
    run += v[k];
  }
}

// -------------------------------------------------------------- 3. sort
// Bucket sort of the W x n digit codes without global atomics:
//   k_sort_hist    per block of ppt x 1024 points: signed digits of all windows,
//                  stored window-major as 2 B codes (c <= 16) or 4 B, and an LDS
//                  histogram over (window, coarse bin), coarse = slot >> FB;
//                  the block histogram goes to bh[(w*NCB+cb)*nblk + blk] so one
//                  exclusive scan of bh yields every block's output position.
//   k_sort_coarse  block (blk, w): LDS-ranked, LDS-staged scatter of its codes
//                  into the coarse segments (runs of consecutive addresses).
//                  Entries are 4 B (fine | sign | index) when the point index
//                  fits, else 8 B.  (Recomputing the digits here instead of
//                  storing them was measured slower: profiles/r01_s2.)
//   k_sort_fine    block per (w, cb) segment: LDS counting sort on the FB fine
//                  bits, the segment cached in LDS between the two passes;
//                  writes the bucket offsets and sorted[] (index | sign << 31).
// Traffic per scalar at c = 16 (W = 16): 32 B read, 32 B digits written and
// read, 64 B entries written and read once, 64 B sorted written (~290 B; was
// ~600 B with 4-B digits, 8-B entries and two global passes in k_sort_fine).
constexpr int kSortThreads = 1024;
constexpr int kSortPerThread = 8;                      // max points per thread (SortGeom::ppt)
constexpr int kSortB = kSortThreads * kSortPerThread;  // max points per block (fixed-base padding)
constexpr uint32_t kFineChunkBytes = 32768;            // auto: chunk buffer of segments larger than one chunk
constexpr size_t kMaxLds = 160 * 1024;                 // LDS per CU (one workgroup may take all of it)
#ifndef PM_FINE_THREADS  // A/B builds only: 256 / 1024 measured slower (profiles/r03/sort_fine/fine_threads.jsonl)
#define PM_FINE_THREADS 512
#endif
constexpr int kFineThreads = PM_FINE_THREADS;

struct SortGeom {
  int FB;    // fine bits
  int NCB;   // coarse bins per window
  int nblk;  // point blocks of ppt * kSortThreads points
  int blk0;  // k_sort_hist: first block of this launch (chunked launches behind a chunked scalar copy)
  int ppt;   // points per thread, <= kSortPerThread
  int hsub;  // coarse geometry: histogram blocks per coarse block (bofs rows hold nblk histogram blocks)
  // words the histogram kernel zeroes for later stages (instead of two
  // hipMemsetAsync fills per call): the scan sentinel, and the chain-list
  // counters (4 words) of each window group
  uint32_t* clr_bh;
  uint32_t* clr_longs;
  uint32_t clr_stride;  // words between group headers
  int clr_groups;
  // entry index remap of k_sort_coarse (a part of a row table's points, the
  // split scalar copy): sort-row entry e = j rstride + i -> table index
  // e + j rdelta + roff (= j npad + c0 + i); rdelta = roff = 0: e itself
  uint32_t rstride, rdelta, roff;
};

// signed digit of window w (WinGeom), carry in/out; returns |d| | neg << 31
// (0 = no contribution).  The top window never carries (scalars < 2^255).
template <int W, class Fs>
__device__ __forceinline__ uint32_t signed_digit(const Fe<Fs>& s, int w, uint32_t& carry) {
  using G = WinGeom<W>;
  const int C = G::width(w);
  const int bit = G::offset(w);
  const int limb = bit >> 5, sh = bit & 31;
  const uint32_t lo = s.l[limb] >> sh;
  const uint32_t hi = (sh != 0 && limb + 1 < 8) ? (s.l[limb + 1] << (32 - sh)) : 0u;
  const uint32_t raw = (lo | hi) & ((1u << C) - 1u);
  uint32_t d = raw + carry;
  uint32_t neg = 0;
  if (w != W - 1 && d > (1u << (C - 1))) {
    d = (1u << C) - d;
    neg = 1;
    carry = 1;
  } else {
    carry = 0;
  }
  return d ? (d | (neg << 31)) : 0u;
}

template <class Fs>
__device__ __forceinline__ Fe<Fs> load_canonical(const uint32_t* scalars, uint32_t i, uint32_t canonical) {
  Fe<Fs> s = load_fe4<Fs>(reinterpret_cast<const uint4*>(scalars + 8ull * i));
  return canonical ? s : fe_from_mont<Fs>(s);
}

__device__ __forceinline__ void sort_clear(const SortGeom& g) {
  if (threadIdx.x == 0 && g.clr_bh) *g.clr_bh = 0u;
  if (threadIdx.x < 4u * (uint32_t)g.clr_groups)
    g.clr_longs[(threadIdx.x >> 2) * g.clr_stride + (threadIdx.x & 3u)] = 0u;
}

// stored digit: D16 (cmax <= 16): (|d| - 1) | neg << 15, 0xFFFF = zero
// (|d| = 2^15 only occurs positive, so that code is free); else |d| | neg << 31
template <bool D16>
struct DigitCode;
template <>
struct DigitCode<true> {
  using T = uint16_t;
  static __device__ __forceinline__ T enc(uint32_t code) {
    return code ? (uint16_t)(((code & ~kNegBit) - 1u) | ((code >> 31) << 15)) : (uint16_t)0xFFFFu;
  }
  static __device__ __forceinline__ uint32_t dec(T v) {
    return v == 0xFFFFu ? 0u : (((uint32_t)v & 0x7FFFu) + 1u) | (((uint32_t)v >> 15) << 31);
  }
};
template <>
struct DigitCode<false> {
  using T = uint32_t;
  static __device__ __forceinline__ T enc(uint32_t code) { return code; }
  static __device__ __forceinline__ uint32_t dec(T v) { return v; }
};

// stride: digit row length (n, or the fixed-base table's padded length with
// zero codes written for i in [n, stride)); kmerge: windows w, w + Wr, ...
// (Wr = W / kmerge) share bucket set r = w mod Wr: window w's digits go to
// digit row r * kmerge + j (j = w / Wr) and its histogram rows are laid out
// (r, coarse bin, j, block), so sort row r is the kmerge digit rows of set r
// back to back and entry j * stride + i is table point (j, i) = [2^{o_{j Wr}}] P_i
// (kmerge = 1: plain windows; kmerge = W: the fixed-base MSM's one bucket set).
template <class Fs, int W, bool D16>
__global__ void __launch_bounds__(kSortThreads) k_sort_hist(const uint32_t* __restrict__ scalars, uint32_t n,
                                                            uint32_t canonical, SortGeom g,
                                                            typename DigitCode<D16>::T* __restrict__ digits,
                                                            uint32_t* __restrict__ bh, uint32_t stride,
                                                            uint32_t kmerge) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];  // W * NCB
  const int nbins = W * g.NCB;
  const uint32_t Wr = (uint32_t)W / kmerge;
  const uint32_t blk = blockIdx.x + (uint32_t)g.blk0;
  if (blk == 0) sort_clear(g);
  for (int k = threadIdx.x; k < nbins; k += kSortThreads) hist[k] = 0;
  __syncthreads();
  // the next point's scalar is loaded while this one is digitised
  const uint32_t ib = blk * g.ppt * kSortThreads + threadIdx.x;
  Fe<Fs> nx;
  if (ib < n) nx = load_fe4<Fs>(reinterpret_cast<const uint4*>(scalars + 8ull * ib));
  for (int r = 0; r < g.ppt; r++) {
    const uint32_t i = ib + (uint32_t)r * kSortThreads;
    if (i >= stride) break;
    if (i >= n) {
#pragma unroll
      for (int w = 0; w < W; w++)
        digits[(size_t)((w % Wr) * kmerge + w / Wr) * stride + i] = DigitCode<D16>::enc(0u);
      continue;
    }
    const Fe<Fs> raw = nx;
    if (r + 1 < g.ppt && i + kSortThreads < n)
      nx = load_fe4<Fs>(reinterpret_cast<const uint4*>(scalars + 8ull * (i + kSortThreads)));
    const Fe<Fs> s = canonical ? raw : fe_from_mont<Fs>(raw);
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint32_t code = signed_digit<W, Fs>(s, w, carry);
      digits[(size_t)((w % Wr) * kmerge + w / Wr) * stride + i] = DigitCode<D16>::enc(code);
      if (code) atomicAdd(&hist[w * g.NCB + ((code & ~kNegBit) >> g.FB)], 1u);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nbins; k += kSortThreads) {
    const uint32_t w = k / g.NCB, cb = k - w * g.NCB;
    const uint32_t row = ((w % Wr) * (uint32_t)g.NCB + cb) * kmerge + w / Wr;
    bh[tile_index(scan_tiles((uint32_t)nbins, (uint32_t)g.nblk), row, blk)] = hist[k];
  }
}

// coarse-segment entry: WIDE = slot << 32 | index | sign << 31;
// narrow = fine << (32 - FB) | sign << (31 - FB) | index  (index < 2^(31 - FB))
template <bool WIDE>
struct SortEntry;
template <>
struct SortEntry<true> {
  using T = uint64_t;
  static __device__ __forceinline__ T make(uint32_t slot, uint32_t i, uint32_t neg, int) {
    return ((uint64_t)slot << 32) | (i | (neg << 31));
  }
  static __device__ __forceinline__ uint32_t fine(T v, uint32_t fmask, int) { return (uint32_t)(v >> 32) & fmask; }
  static __device__ __forceinline__ uint32_t code(T v, int) { return (uint32_t)v; }
};
template <>
struct SortEntry<false> {
  using T = uint32_t;
  static __device__ __forceinline__ T make(uint32_t slot, uint32_t i, uint32_t neg, int FB) {
    const uint32_t fm = (1u << FB) - 1u;
    return (FB ? ((slot & fm) << (32 - FB)) : 0u) | (neg << (31 - FB)) | i;
  }
  static __device__ __forceinline__ uint32_t fine(T v, uint32_t, int FB) { return FB ? v >> (32 - FB) : 0u; }
  static __device__ __forceinline__ uint32_t code(T v, int FB) {
    const uint32_t imask = (1u << (31 - FB)) - 1u;
    return (v & imask) | (((v >> (31 - FB)) & 1u) << 31);
  }
};

// block (blk = blockIdx.x, w = blockIdx.y) of PPT x kSortThreads points.
// PPT is a template parameter: with g.ppt read at run time the kernel ran
// ~45% slower at the same geometry (0.069 vs 0.047 ms at 2^20).
// Each lane takes PPT consecutive codes with one vector load (when the row is
// aligned for it); the block's global bin starts are read once into LDS
// (round 2 loaded bofs[] per entry in the write-out loop).
template <int PPT, class DT>
__device__ __forceinline__ void load_codes(const DT* __restrict__ row, uint32_t i0, uint32_t n, bool vec,
                                           uint32_t (&code)[PPT]) {
  constexpr int bytes = PPT * (int)sizeof(DT);
  if (vec && i0 + PPT <= n && (bytes == 16 || bytes == 8 || bytes == 4)) {
    DT v[PPT];
    if constexpr (bytes == 16) {
      *reinterpret_cast<uint4*>(v) = *reinterpret_cast<const uint4*>(row + i0);
    } else if constexpr (bytes == 8) {
      *reinterpret_cast<uint2*>(v) = *reinterpret_cast<const uint2*>(row + i0);
    } else if constexpr (bytes == 4) {
      *reinterpret_cast<uint32_t*>(v) = *reinterpret_cast<const uint32_t*>(row + i0);
    }
#pragma unroll
    for (int r = 0; r < PPT; r++) code[r] = DigitCode<sizeof(DT) == 2>::dec(v[r]);
  } else if (vec && i0 + PPT <= n && bytes == 32) {
    DT v[PPT];
    reinterpret_cast<uint4*>(v)[0] = reinterpret_cast<const uint4*>(row + i0)[0];
    reinterpret_cast<uint4*>(v)[1] = reinterpret_cast<const uint4*>(row + i0)[1];
#pragma unroll
    for (int r = 0; r < PPT; r++) code[r] = DigitCode<sizeof(DT) == 2>::dec(v[r]);
  } else {
#pragma unroll
    for (int r = 0; r < PPT; r++) code[r] = i0 + r < n ? DigitCode<sizeof(DT) == 2>::dec(row[i0 + r]) : 0u;
  }
}
template <bool D16, bool WIDE, int PPT>
__global__ void __launch_bounds__(kSortThreads) k_sort_coarse(const typename DigitCode<D16>::T* __restrict__ digits,
                                                              uint32_t n, SortGeom g,
                                                              const uint32_t* __restrict__ bofs,
                                                              typename SortEntry<WIDE>::T* __restrict__ mid) {
  using E = SortEntry<WIDE>;
  using T = typename E::T;
  using DT = typename DigitCode<D16>::T;
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  constexpr uint32_t sortb = (uint32_t)PPT * kSortThreads;
  T* stage = reinterpret_cast<T*>(sm);                                        // sortb entries
  uint16_t* stage_cb = reinterpret_cast<uint16_t*>(stage + sortb);           // sortb coarse bins
  uint32_t* cnt = reinterpret_cast<uint32_t*>(stage_cb + sortb);             // NCB
  uint32_t* lstart = cnt + g.NCB;                                            // NCB + 1
  uint32_t* scan_tmp = lstart + g.NCB + 1;                                   // kSortThreads/64 + 1
  const uint32_t w = blockIdx.y, blk = blockIdx.x;
  // the block's entries lie in one digit row j (sortb divides rstride)
  const uint32_t remap = (g.rdelta | g.roff) ? blk * sortb / g.rstride * g.rdelta + g.roff : 0u;
  for (int k = threadIdx.x; k < g.NCB; k += kSortThreads) cnt[k] = 0;
  __syncthreads();
  const DT* row = digits + (size_t)w * n;
  // vector loads need the row start aligned to PPT codes (n % PPT == 0 or w == 0)
  const bool vec = (((size_t)w * n) % PPT) == 0;
  const uint32_t i0 = blk * sortb + threadIdx.x * PPT;
  uint32_t code[PPT];
  load_codes<PPT, DT>(row, i0, n, vec, code);
#pragma unroll
  for (int r = 0; r < PPT; r++)
    if (code[r]) atomicAdd(&cnt[(code[r] & ~kNegBit) >> g.FB], 1u);
  __syncthreads();
  uint32_t run = 0;
  for (int base = 0; base < g.NCB; base += kSortThreads) {
    const int k = base + threadIdx.x;
    const uint32_t v = k < g.NCB ? cnt[k] : 0u;
    uint32_t total;
    const uint32_t ex = block_excl_scan(v, scan_tmp, total);
    if (k < g.NCB) lstart[k] = ex + run;
    run += total;
  }
  if (threadIdx.x == 0) lstart[g.NCB] = run;
  __syncthreads();
  const uint32_t nvalid = lstart[g.NCB];
  // cursors; lstart becomes (global start of the bin's run) - (its LDS start)
  for (int k = threadIdx.x; k < g.NCB; k += kSortThreads) {
    const uint32_t ls = lstart[k];
    cnt[k] = ls;
    lstart[k] = bofs[((size_t)w * g.NCB + k) * g.nblk + (size_t)blk * g.hsub] - ls;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < PPT; r++) {
    if (!code[r]) continue;
    const uint32_t slot = code[r] & ~kNegBit;
    const uint32_t cb = slot >> g.FB;
    const uint32_t pos = atomicAdd(&cnt[cb], 1u);
    stage[pos] = E::make(slot, i0 + r + remap, code[r] >> 31, g.FB);
    stage_cb[pos] = (uint16_t)cb;
  }
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < nvalid; e += kSortThreads) mid[lstart[stage_cb[e]] + e] = stage[e];
}

// block per (w, cb) segment; offsets[w*NB + slot] for its slots, sorted[].
// LDS: a segment cache of cache_n entries and a chunk buffer of ch entries.
//   pass 1  the segment is read once with 16-B loads (4 in flight per lane)
//           into the cache while its fine histogram is counted;
//   pass 2  chunk by chunk (ch entries; one chunk when the segment fits the
//           chunk buffer): LDS counting sort of the chunk by fine bits into
//           the chunk buffer, then every fine bin's run goes out to that bin's
//           global cursor, so the stores leave as runs, not scattered 4-B
//           writes (fixed-base 2^23: 3.0 ms of scattered stores before).
// A segment larger than the cache (skewed digits, the fixed-base MSM's merged
// rows at small caches) re-reads each chunk from mid into the cache instead.
template <class T>
__device__ __forceinline__ void fine_entry(T v, T* cache, uint32_t at, uint32_t* hist, uint32_t fmask, int FB) {
  if (cache) cache[at] = v;
  atomicAdd(&hist[SortEntry<sizeof(T) == 8>::fine(v, fmask, FB)], 1u);
}
template <class T>
__device__ __forceinline__ void fine_pass1(const T* __restrict__ mid, uint32_t s0, uint32_t s1, T* cache,
                                           uint32_t* hist, uint32_t fmask, int FB) {
  constexpr uint32_t per = 16 / sizeof(T);  // entries per 16-B load
  constexpr int kUnroll = 4;
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  const uint32_t a0 = min(s1, (s0 + per - 1) & ~(per - 1));
  const uint32_t a1 = max(a0, s1 & ~(per - 1));
  for (uint32_t e = s0 + tid; e < a0; e += nt) fine_entry<T>(mid[e], cache, e - s0, hist, fmask, FB);
  for (uint32_t e = a1 + tid; e < s1; e += nt) fine_entry<T>(mid[e], cache, e - s0, hist, fmask, FB);
  const uint4* v4 = reinterpret_cast<const uint4*>(mid + a0);
  const uint32_t nv = (a1 - a0) / per;
  for (uint32_t k = tid; k < nv; k += kUnroll * nt) {
    uint4 x[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
      if (k + u * nt < nv) x[u] = v4[k + u * nt];
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
      if (k + u * nt >= nv) break;
      const T* ev = reinterpret_cast<const T*>(&x[u]);
      const uint32_t at = a0 - s0 + (k + u * nt) * per;
#pragma unroll
      for (uint32_t q = 0; q < per; q++) fine_entry<T>(ev[q], cache, at + q, hist, fmask, FB);
    }
  }
}
template <bool WIDE>
__global__ void __launch_bounds__(kFineThreads) k_sort_fine(const typename SortEntry<WIDE>::T* __restrict__ mid,
                                                            const uint32_t* __restrict__ bofs, SortGeom g, int W,
                                                            int NB, uint32_t cache_n, uint32_t ch,
                                                            uint32_t* __restrict__ offsets,
                                                            uint32_t* __restrict__ sorted) {
  using E = SortEntry<WIDE>;
  using T = typename E::T;
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int nf = 1 << g.FB;
  T* cache = reinterpret_cast<T*>(sm);                                 // cache_n entries (>= ch)
  T* otmp = cache + cache_n;                                           // ch entries
  uint32_t* hist = reinterpret_cast<uint32_t*>(otmp + ch);             // nf global cursors
  uint32_t* lcur = hist + nf;                                          // nf chunk cursors
  uint32_t* lst = lcur + nf;                                           // nf chunk starts
  uint32_t* scan_tmp = lst + nf;                                       // kFineThreads/64 + 1
  const uint32_t seg = blockIdx.x;     // = w * NCB + cb
  const uint32_t w = seg / g.NCB, cb = seg - w * g.NCB;
  const uint32_t s0 = bofs[(size_t)seg * g.nblk];
  const uint32_t s1 = bofs[(size_t)(seg + 1) * g.nblk];  // next segment (or total)
  const bool cached = s1 - s0 <= cache_n;
  const uint32_t fmask = (uint32_t)nf - 1u;
  for (int k = threadIdx.x; k < nf; k += kFineThreads) hist[k] = 0;
  __syncthreads();
  fine_pass1<T>(mid, s0, s1, cached ? cache : nullptr, hist, fmask, g.FB);
  __syncthreads();
  // exclusive scan of the fine histogram: bucket offsets and global cursors
  uint32_t run = 0;
  for (int base = 0; base < nf; base += kFineThreads) {
    const int k = base + threadIdx.x;
    const uint32_t v = k < nf ? hist[k] : 0u;
    uint32_t total;
    const uint32_t ex = block_excl_scan(v, scan_tmp, total);
    if (k < nf) {
      const uint32_t slot = (cb << g.FB) + k;
      hist[k] = s0 + ex + run;
      if (slot < (uint32_t)NB) offsets[(size_t)w * NB + slot] = s0 + ex + run;
    }
    run += total;
  }
  // slots beyond the coarse range (window padding) and the final sentinel
  if (cb == (uint32_t)g.NCB - 1) {
    for (uint32_t slot = ((uint32_t)g.NCB << g.FB) + threadIdx.x; slot < (uint32_t)NB; slot += kFineThreads)
      offsets[(size_t)w * NB + slot] = s1;
    if (threadIdx.x == 0 && w == (uint32_t)W - 1) offsets[(size_t)W * NB] = s1;
  }
  __syncthreads();
  for (uint32_t c0 = s0; c0 < s1; c0 += ch) {
    const uint32_t m = min(ch, s1 - c0);
    const T* src = cached ? cache + (c0 - s0) : cache;
    for (int k = threadIdx.x; k < nf; k += kFineThreads) lcur[k] = 0;
    __syncthreads();
    if (cached) {
      for (uint32_t e = threadIdx.x; e < m; e += kFineThreads) atomicAdd(&lcur[E::fine(src[e], fmask, g.FB)], 1u);
    } else {
      fine_pass1<T>(mid, c0, c0 + m, cache, lcur, fmask, g.FB);  // stage the chunk (16-B loads)
    }
    __syncthreads();
    uint32_t lrun = 0;
    for (int base = 0; base < nf; base += kFineThreads) {
      const int k = base + threadIdx.x;
      const uint32_t v = k < nf ? lcur[k] : 0u;
      uint32_t total;
      const uint32_t ex = block_excl_scan(v, scan_tmp, total);
      if (k < nf) {
        lst[k] = ex + lrun;
        lcur[k] = ex + lrun;
      }
      lrun += total;
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < m; e += kFineThreads) {
      const T v = src[e];
      otmp[atomicAdd(&lcur[E::fine(v, fmask, g.FB)], 1u)] = v;
    }
    __syncthreads();
    // runs of one fine bin are consecutive in otmp and in sorted[]
    for (uint32_t j = threadIdx.x; j < m; j += kFineThreads) {
      const T v = otmp[j];
      const uint32_t b = E::fine(v, fmask, g.FB);
      sorted[hist[b] + (j - lst[b])] = E::code(v, g.FB);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nf; k += kFineThreads) hist[k] += lcur[k] - lst[k];
    __syncthreads();
  }
}

// ----------------------------------------------------------- 4. accumulate
// One launch covers every bucket set: the sorted positions [offsets[0],
// offsets[s1]) with s1 = Wr * NB.  Slice t covers positions [t*chunk, ...).
// A bucket is *owned* by the slice holding its first element; the owner
// writes its (possibly partial) sum to buckets[]; a slice whose first bucket
// started in an earlier slice writes that partial to head[t], and
// k_bucket_seg_q folds the chain buckets[gb] + head[t_first + 1 ..] of every
// bucket (found from the offsets alone, so this kernel queues nothing).
__device__ __forceinline__ uint32_t find_bucket(const uint32_t* __restrict__ offsets, uint32_t lo, uint32_t hi,
                                                uint32_t pos) {
  // largest gb in [lo, hi) with offsets[gb] <= pos
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= pos) lo = mid; else hi = mid;
  }
  return lo;
}

// Chains up to kSerialChain later slices are folded by the bucket's own lane
// in k_bucket_seg_q; longer ones (giant buckets: adversarial or highly
// repetitive scalars, e.g. many scalars equal to 1) by the whole wave, one
// chain at a time (a strided sum over 64 lanes and a butterfly), when that
// beats the lane's own walk.  (A cut at 8 slices sent the fixed-base MSM's
// merged buckets, ~8-9 slices each, wave-wide: 2^20 k_bucket_seg_q 0.05 ->
// 1.29 ms, gpurun_out/b of round 3.)
constexpr uint32_t kSerialChain = 32;

// Base gather by LDS-DMA one entry ahead: global_load_lds writes the next
// entry's 64-B base straight into LDS (no VGPRs held across the addition), so
// its L2 / Infinity Cache latency hides behind this entry's mixed addition.
// Per wave 4 KiB: [16-B chunk][lane].  (The plain register-load form measured
// slower at every size, round 2: profiles/r02/xp/.)
__device__ __forceinline__ void glds_base(const uint32_t* g, uint4* lds_wave) {
#pragma unroll
  for (int k = 0; k < 4; k++)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + 4 * k),
                                     (__attribute__((address_space(3))) void*)(lds_wave + 64 * k), 16, 0, 0);
}
#ifndef PM_ACC_WAVES
#define PM_ACC_WAVES 4  // waves per SIMD the register budget is sized for
#endif
template <class F>
__global__ void __launch_bounds__(256, PM_ACC_WAVES) k_accumulate(const uint32_t* __restrict__ sorted,
                                                    const uint32_t* __restrict__ offsets, uint32_t s1,
                                                    const uint32_t* __restrict__ bases, uint32_t chunk,
                                                    Xyzz<F>* __restrict__ buckets,
                                                    Xyzz<F>* __restrict__ head) {
  __shared__ uint4 sb[4 * 4 * 64];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t base = offsets[0], total = offsets[s1];
  const uint32_t start = base + t * chunk;
  if (start >= total) return;
  const uint32_t end = min(start + chunk, total);
  uint32_t gb = find_bucket(offsets, 0, s1, start);
  uint32_t bend = offsets[gb + 1];
  bool owned = offsets[gb] == start;
  // acc is empty ("fresh") at a bucket start and after a cancellation; an
  // empty acc has ZZ = 0, so it stores as the identity
  Xyzz29<F> acc = xyzz29_inf<F>();
  bool fresh = true;
  uint32_t code = sorted[start], nxt = 0;  // code = entry p (base in LDS), nxt = entry p + 1
  uint4* sw = sb + 256 * (threadIdx.x >> 6);
  const uint32_t ln = threadIdx.x & 63;
  glds_base(bases + 16ull * (code & ~kNegBit), sw);
  if (start + 1 < end) nxt = sorted[start + 1];
  for (uint32_t p = start; p < end; p++) {
    F29<F> x, y;
    const uint32_t ccode = code;
    {
      // this entry's base landed in LDS (vmcnt covers LDS-DMA; everything
      // outstanding was issued before the previous addition); read it, and
      // only then (lgkmcnt) let the next entry's DMA overwrite the slots
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      const uint4 a = sw[ln], b = sw[64 + ln], c = sw[128 + ln], d = sw[192 + ln];
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      const uint32_t wx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const uint32_t wy[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
      x = f29_unpack<F>(wx);
      y = f29_unpack<F>(wy);
    }
    if (p == bend) {
      // the next bucket's end is loaded before the store, so its use waits
      // for the load only (vmcnt counts stores too)
      const uint32_t nb = offsets[gb + 2];
      store_xyzz29<F>(owned ? &buckets[gb] : &head[t], xyzz29_settle<F>(acc));
      fresh = true;
      acc.ZZ = f29_zero<F>();
      gb++;
      bend = nb;
      // skip empty buckets by binary search: a window narrower than cmax
      // leaves half its slots empty, and a linear walk over them (one
      // dependent load each) stalled the lane crossing into the next window
      // (W = 18 at 2^20: accumulate 1.06 -> 2.0 ms)
      if (bend <= p) {
        gb = find_bucket(offsets, gb, s1, p);
        bend = offsets[gb + 1];
      }
      owned = true;
    }
    if (p + 1 < end) {
      glds_base(bases + 16ull * (nxt & ~kNegBit), sw);
      code = nxt;
      if (p + 2 < end) nxt = sorted[p + 2];
    }
    // identity base (0, 0): y = 0 holds for no point of odd order
    if (f29_is_zero_exact<F>(y)) continue;
    const uint32_t negm = 0u - (ccode >> 31);  // kNegBit
    Xyzz29<F> r = xyzz29_madd_lazy<F>(acc, x, y, negm);
    // ZZ3 = 0 mod p only when acc = +-point: the filter almost never hits,
    // and the wave-uniform branch keeps the exact check off the hot path
    const bool hit = !fresh && f29_zero_filter<F>(r.ZZ);
    if (fresh) {  // first point of the bucket (divergent, every few entries)
      r.X = x;
      r.Y = negm ? f29_neg_canon<F>(y) : y;
      r.ZZ = f29_const<F>(F29Consts<F>::ONE);
      r.ZZZ = r.ZZ;
      fresh = false;
    }
    if (__builtin_amdgcn_ballot_w64(hit)) {
      if (hit) fresh = xyzz29_madd_fix<F>(r, x, y, negm);
    }
    acc = r;
  }
  store_xyzz29<F>(owned ? &buckets[gb] : &head[t], xyzz29_settle<F>(acc));
}

// Base conversion (once per MSM): Rust-layout R = 2^256 Montgomery -> the
// radix-2^29 pipeline's R = 2^261 form, canonical, same packed 64-B layout.
template <class F>
__global__ void __launch_bounds__(256) k_bases_to_r261(const uint32_t* __restrict__ in, uint32_t n,
                                                       uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4* q = reinterpret_cast<const uint4*>(in + 16ull * i);
  uint4* o = reinterpret_cast<uint4*>(out + 16ull * i);
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const uint4 a = q[2 * c], b = q[2 * c + 1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    st29<F>(o + 2 * c, f29_canon<F>(f29_from_r256<F>(w)));
  }
}

// Fixed-base table (pm_fixed_bases_create*): entry (j, i) at j * npad + i is
// [2^{o_{j Wr}}] P_i (Wr = W / rows) as a canonical affine point in the
// pipeline's R = 2^261 form, o_w the bit offset of window w (WinGeom).  One
// lane per base: repeated XYZZ doublings, one inversion per row.  Identity
// bases and the padding rows [n, npad) stay (0, 0), which k_accumulate skips.
template <class F>
__global__ void __launch_bounds__(256) k_fixed_table(const uint32_t* __restrict__ in, uint32_t n, uint32_t npad,
                                                     int W, int base, int extra, int rows,
                                                     uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npad) return;
  F29<F> x = f29_zero<F>(), y = f29_zero<F>();
  bool ident = true;
  if (i < n) {
    const uint4* q = reinterpret_cast<const uint4*>(in + 16ull * i);
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    const uint32_t wx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t wy[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
    uint32_t z = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) z |= wx[k] | wy[k];
    ident = z == 0;
    if (!ident) {
      x = f29_canon<F>(f29_from_r256<F>(wx));
      y = f29_canon<F>(f29_from_r256<F>(wy));
    }
  }
  uint4* o = reinterpret_cast<uint4*>(out + 16ull * i);
  st29<F>(o, x);
  st29<F>(o + 2, y);
  if (ident) {
    for (int j = 1; j < rows; j++) {
      uint4* ow = reinterpret_cast<uint4*>(out + 16ull * ((size_t)j * npad + i));
      st29<F>(ow, x);
      st29<F>(ow + 2, y);
    }
    return;
  }
  bool acc_inf = true;
  Xyzz29<F> acc = xyzz29_madd<F>(xyzz29_inf<F>(), x, y, acc_inf);
  const int Wr = W / rows;
  for (int j = 1; j < rows; j++) {
    int steps = 0;  // o_{j Wr} - o_{(j-1) Wr}: the widths of windows (j-1) Wr .. j Wr - 1
    for (int w = (j - 1) * Wr; w < j * Wr; w++) steps += base + (w < extra ? 1 : 0);
    for (int k = 0; k < steps; k++) acc = xyzz29_dbl<F>(acc);  // P has odd prime order: never the identity
    F29<F> ax, ay;
    xyzz29_to_aff<F>(acc, ax, ay);
    uint4* ow = reinterpret_cast<uint4*>(out + 16ull * ((size_t)j * npad + i));
    st29<F>(ow, ax);
    st29<F>(ow + 2, ay);
  }
}

// ------------------------------------------- 5. chains and segment sums
// One quad per segment of kSegQ = 4 buckets: lane q folds bucket q's
// slice-boundary chain (buckets[gb] plus head[t] of every later slice the
// bucket reaches), then the quad shares the four sums and computes S = B0 +
// B1 + B2 + B3 and T = B1 + 2 B2 + 3 B3 with quad-cooperative additions
// (coop29.hpp).  A chain of more than kSerialChain slices (a giant bucket)
// is folded by the whole wave instead: the lanes stride over its partials,
// a butterfly sums the 64 results, and the owning lane adds them -- so no
// separate long-chain launch (round 2: k_fixup_long, ~5 us per MSM, almost
// always empty) and no chain list from k_accumulate.
constexpr uint32_t kSegQ = 4;  // buckets per segment: a quad (= kL1, runtime.hpp)
template <int K, class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_qbc(const Xyzz29<F>& p) {  // lane K's point, quad-wide
  return Xyzz29<F>{qbc<K, F>(p.X), qbc<K, F>(p.Y), qbc<K, F>(p.ZZ), qbc<K, F>(p.ZZZ)};
}
template <class F>
__device__ __forceinline__ F29<F> f29_shfl_xor(const F29<F>& v, int m) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = (uint32_t)__shfl_xor((int)v.l[i], m, 64);
  return r;
}
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_shfl_xor(const Xyzz29<F>& p, int m) {
  return Xyzz29<F>{f29_shfl_xor<F>(p.X, m), f29_shfl_xor<F>(p.Y, m), f29_shfl_xor<F>(p.ZZ, m),
                   f29_shfl_xor<F>(p.ZZZ, m)};
}
// lane k of a quad stores coordinate k of p (Norm, < 4p) converted to the
// Rust R = 2^256 layout into *dst (the host Horner's term format)
template <class F>
__device__ __forceinline__ void store_r256_q(Xyzz<F>* dst, const Xyzz29<F>& p, uint32_t lk) {
  const F29<F> c = qsel<F>(lk, p.X, p.Y, p.ZZ, p.ZZZ);
  uint32_t o[8];
  f29_to_r256<F>(c, o);
  uint4* q = reinterpret_cast<uint4*>(dst);
  q[2 * lk] = make_uint4(o[0], o[1], o[2], o[3]);
  q[2 * lk + 1] = make_uint4(o[4], o[5], o[6], o[7]);
}
// Segments cover slots [0, K) (M1 = K / kSegQ); the top bucket K is folded
// by lane 0 of segment 0 instead of slot 0 (digit 0 has no bucket, and
// whatever slot 0 holds has weight 0: S_0 enters no bit sum, T_0 weighs lane 0
// by 0); that quad converts it and stores it as the set's last host term,
// Q[w * NQ + NQ - 1].
// One sorted list's share of a bucket (the split scalar copy sorts and
// accumulates two parts of the points separately, engine.hpp): its partial in
// buckets[slot] when the bucket has entries in that list, plus the chain
// head[t_first + 1 .. t_last] of the later slices it reaches.
template <class F>
struct SegChunk {
  const uint32_t* offsets;
  uint32_t chunk, nthreads;
  const Xyzz<F>* buckets;
  const Xyzz<F>* head;
};
// adds chunk c's share of bucket `slot` to B (first: B is still empty)
template <class F, bool FIRST>
__device__ __forceinline__ void seg_fold_chunk(const SegChunk<F>& c, bool valid, size_t slot, Xyzz29<F>& B) {
  const uint32_t base = c.offsets[0];
  const uint32_t bs = valid ? c.offsets[slot] : 0u, be = valid ? c.offsets[slot + 1] : 0u;
  uint32_t tf = 0, tl = 0;
  if (bs != be) {
    const Xyzz29<F> b0 = load_xyzz29<F>(&c.buckets[slot]);
    B = FIRST ? b0 : xyzz29_add<F>(B, b0);
    tf = (bs - base) / c.chunk;
    tl = min((be - 1 - base) / c.chunk, c.nthreads - 1);
    if (tl - tf <= kSerialChain)
      for (uint32_t t = tf + 1; t <= tl; t++) B = xyzz29_add<F>(B, load_xyzz29<F>(&c.head[t]));
  }
  // giant buckets: the wave folds each long chain in turn (wave-uniform loop)
  uint64_t lm = __ballot(tl - tf > kSerialChain);
  const uint32_t ln = __lane_id();
  if (lm) {
    // wave-wide only while it beats the lanes' own walks: ~ceil(len / 64) + 6
    // additions per chain, one chain after another, against the longest
    // chain's len serial additions (64 adjacent 100-slice buckets: serial;
    // one 10^4-slice bucket: wave-wide)
    uint32_t mx = tl - tf;
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, m, 64));
    uint32_t coop = 0;
    for (uint64_t r = lm; r; r &= r - 1) coop += (mx + 63) / 64 + 6;
    if (mx <= kSerialChain + coop) {
      if (tl - tf > kSerialChain)
        for (uint32_t t = tf + 1; t <= tl; t++) B = xyzz29_add<F>(B, load_xyzz29<F>(&c.head[t]));
      lm = 0;
    }
  }
  while (lm) {
    const int L = __ffsll((unsigned long long)lm) - 1;
    lm &= lm - 1;
    const uint32_t a = (uint32_t)__shfl((int)tf, L, 64) + 1u, z = (uint32_t)__shfl((int)tl, L, 64);
    Xyzz29<F> cs = xyzz29_inf<F>();
    for (uint32_t t = a + ln; t <= z; t += 64) cs = xyzz29_add<F>(cs, load_xyzz29<F>(&c.head[t]));
#pragma unroll 1
    for (int m = 32; m > 0; m >>= 1) cs = xyzz29_add<F>(cs, xyzz29_shfl_xor<F>(cs, m));
    if (ln == (uint32_t)L) B = xyzz29_add<F>(B, cs);
  }
}
// the sorted lists of one MSM: 1, or the split scalar copy's parts
constexpr int kMaxParts = 3;
template <class F>
struct SegChunks {
  SegChunk<F> c[kMaxParts];
};
// NCH > 1: the bucket sums of the split copy's NCH sorted lists
template <class F, int NCH>
__global__ void __launch_bounds__(256, 2) k_bucket_seg_q(SegChunks<F> cs, int Wr, int NB, uint32_t M1,
                                                      Xyzz<F>* __restrict__ S, Xyzz<F>* __restrict__ T,
                                                      Xyzz<F>* __restrict__ Q, int NQ) {
  const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = gl >> 2, q = gl & 3u;
  // lanes past the last segment stay (inactive values) for the wave-wide fold
  const bool valid = g < (uint32_t)Wr * M1;
  const uint32_t w = valid ? g / M1 : 0u, j = valid ? g - w * M1 : 1u;
  const bool top = valid && j == 0 && q == 0;
  const size_t slot = (size_t)w * NB + (top ? M1 * kSegQ : j * kSegQ + q);
  Xyzz29<F> B = xyzz29_inf<F>();
  seg_fold_chunk<F, true>(cs.c[0], valid, slot, B);
#pragma unroll
  for (int k = 1; k < NCH; k++) seg_fold_chunk<F, false>(cs.c[k], valid, slot, B);
  // broadcast each lane's sum only when it is consumed (fewer live points)
  const Xyzz29<F> B3 = xyzz29_qbc<3, F>(B);
  const Xyzz29<F> p23 = xyzz29_add_q<F>(xyzz29_qbc<2, F>(B), B3);
  const Xyzz29<F> p123 = xyzz29_add_q<F>(xyzz29_qbc<1, F>(B), p23);
  const Xyzz29<F> tv = xyzz29_add_q<F>(xyzz29_add_q<F>(p123, p23), B3);
  const Xyzz29<F> sv = xyzz29_add_q<F>(xyzz29_qbc<0, F>(B), p123);
  if (!valid) return;
  if (q == 0) store_xyzz29<F>(&S[g], sv);
  if (q == 1) store_xyzz29<F>(&T[g], tv);
  if (j == 0) store_r256_q<F>(&Q[(size_t)w * NQ + NQ - 1], xyzz29_qbc<0, F>(B), q);
}

// ------------------------------------------------------ 6. bit sums
// block (job, w, z): job < NB2 -> G_job = sum_{j : (j >> job) & 1} S_j
// (only the j with that bit set are enumerated, so no lane idles); job >= NB2
// -> partial sum of T_j over part (job - NB2) of kTJobs equal ranges.
// kRedThreads lanes: strided partial sums, then an LDS tree.  With nsplit > 1
// (few bucket sets, e.g. the row tables' 4 or the fixed-base MSM's one)
// nsplit blocks share a job: each reduces every nsplit-th stride, parks its
// partial in P, and the last block to finish (atomic ticket) folds the
// nsplit partials with log2(nsplit) quad-cooperative levels (round 2 ran a
// fixed 6-level plain tree here, i.e. four wasted addition latencies at
// nsplit = 4).  The result goes out converted to the Rust R = 2^256 layout
// as host term Q[w * NQ + job] (round 2 folded pairs of bit sums and
// converted them in a separate k_bits_combine launch, ~19 us per MSM).
constexpr int kRedThreads = 512;
constexpr int kTJobs = 2;
constexpr int kMaxSplit = 64;
// reduce lds[0 .. count) (count a power of two <= kRedThreads; acc = this
// lane's lds[tid]) into lds[0]; quad-cooperative once 4 s lanes are free
template <class F>
__device__ __forceinline__ void lds_tree(Xyzz29<F>* lds, int count, Xyzz29<F> acc) {
  const int tid = threadIdx.x;
  for (int s = count / 2; s > 0; s >>= 1) {
    if (4 * s <= (int)blockDim.x) {
      const int v = tid >> 2;
      if (v < s) {
        const Xyzz29<F> r = xyzz29_add_q<F>(lds[v], lds[v + s]);
        if ((tid & 3) == 0) lds[v] = r;  // the quad read lds[v] in this same wave
      }
    } else if (tid < s) {
      acc = xyzz29_add<F>(acc, lds[tid + s]);
      lds[tid] = acc;
    }
    __syncthreads();
  }
}
template <class F>
__global__ void __launch_bounds__(kRedThreads) k_bucket_bits(const Xyzz<F>* __restrict__ S,
                                                             const Xyzz<F>* __restrict__ T, int M1, int NB2,
                                                             Xyzz<F>* __restrict__ Q, int NQ, int nsplit,
                                                             Xyzz<F>* __restrict__ P, uint32_t* __restrict__ tickets) {
  __shared__ Xyzz29<F> lds[kRedThreads];
  __shared__ uint32_t last;
  const int w = blockIdx.y, job = blockIdx.x, tid = threadIdx.x, z = blockIdx.z;
  const int lane = z * kRedThreads + tid, stride = kRedThreads * nsplit;
  Xyzz29<F> acc = xyzz29_inf<F>();
  if (job < NB2) {
    const int low = (1 << job) - 1;
    for (int m = lane;; m += stride) {
      const int j = ((m & ~low) << 1) | (1 << job) | (m & low);  // m-th index with bit `job` set
      if (j >= M1) break;
      acc = xyzz29_add<F>(acc, load_xyzz29<F>(&S[(size_t)w * M1 + j]));
    }
  } else {
    const int per = (M1 + kTJobs - 1) / kTJobs;
    const int j0 = (job - NB2) * per, j1 = min(M1, j0 + per);
    for (int j = j0 + lane; j < j1; j += stride) acc = xyzz29_add<F>(acc, load_xyzz29<F>(&T[(size_t)w * M1 + j]));
  }
  lds[tid] = acc;
  __syncthreads();
  lds_tree<F>(lds, kRedThreads, acc);
  if (nsplit > 1) {
    const size_t out = (size_t)w * (NB2 + kTJobs) + job;
    if (tid == 0) {
      store_xyzz29<F>(&P[out * nsplit + z], lds[0]);
      __threadfence();
      last = atomicAdd(&tickets[out], 1u) == (uint32_t)nsplit - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    int cnt = 1;
    while (cnt < nsplit) cnt <<= 1;
    acc = tid < nsplit ? load_xyzz29<F>(&P[out * nsplit + tid]) : xyzz29_inf<F>();
    __syncthreads();  // every lane has read lds[0] above
    if (tid < cnt) lds[tid] = acc;
    __syncthreads();
    lds_tree<F>(lds, cnt, acc);
    if (tid == 0) tickets[out] = 0;  // ready for the next MSM
  }
  if (tid < 4) store_r256_q<F>(&Q[(size_t)w * NQ + job], lds[0], (uint32_t)tid);
}

// ------------------------------------------------------ synthetic inputs
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t synth_word(uint64_t seed, uint64_t i, uint64_t j) {
  return mix64(mix64(seed + i) + j);
}
// uniform in [0, MOD) (canonical), mirrors oracle/pasta.py synth_scalar
template <class Fs>
__host__ __device__ __forceinline__ Fe<Fs> synth_scalar(uint64_t seed, uint64_t i) {
  for (uint64_t t = 0;; t++) {
    uint64_t w[4];
    for (int k = 0; k < 4; k++) w[k] = synth_word(seed, i, 4 * t + k);
    w[3] &= (Fs::NBITS - 192 >= 64) ? ~0ull : ((1ull << (Fs::NBITS - 192)) - 1ull);
    Fe<Fs> v;
    for (int k = 0; k < 4; k++) {
      v.l[2 * k] = (uint32_t)w[k];
      v.l[2 * k + 1] = (uint32_t)(w[k] >> 32);
    }
    uint32_t br = 0;
    for (int k = 0; k < 8; k++) (void)subb(v.l[k], Fs::MOD[k], br);
    if (br) return v;  // v < MOD
  }
}

template <class Fs>
__global__ void k_synth_scalars(uint64_t seed, uint64_t i0, uint32_t n, uint32_t mont,
                                uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fe<Fs> v = synth_scalar<Fs>(seed, i0 + i);
  if (mont) v = fe_to_mont<Fs>(v);
  store_fe4<Fs>(reinterpret_cast<uint4*>(out + 8ull * i), v);
}

template <class Cv>
__device__ __forceinline__ Aff<typename Cv::Base> generator();

template <>
__device__ __forceinline__ Aff<PallasFp> generator<PallasCurve>() {
  return Aff<PallasFp>{fe_neg<PallasFp>(fe_one<PallasFp>()), fe_add<PallasFp>(fe_one<PallasFp>(), fe_one<PallasFp>())};
}
template <>
__device__ __forceinline__ Aff<VestaFp> generator<VestaCurve>() {
  return Aff<VestaFp>{fe_neg<VestaFp>(fe_one<VestaFp>()), fe_add<VestaFp>(fe_one<VestaFp>(), fe_one<VestaFp>())};
}
template <>
__device__ __forceinline__ Aff<Bn254Fq> generator<Bn254Curve>() {
  return Aff<Bn254Fq>{fe_one<Bn254Fq>(), fe_add<Bn254Fq>(fe_one<Bn254Fq>(), fe_one<Bn254Fq>())};
}

// P = [k]A (k canonical), MSB-first double-and-add
template <class F, class Fs>
__device__ __forceinline__ Xyzz<F> scalar_mul(const Fe<Fs>& k, const Aff<F>& A) {
  Xyzz<F> acc = xyzz_inf<F>();
  for (int i = 7; i >= 0; i--) {
    for (int b = 31; b >= 0; b--) {
      acc = xyzz_dbl<F>(acc);
      if ((k.l[i] >> b) & 1u) acc = xyzz_add_aff<F>(acc, A);
    }
  }
  return acc;
}

// synthetic base i = [a_i]G with a_i = synth_scalar(seed, i) (1 if zero)
template <class Cv>
__global__ void __launch_bounds__(256) k_synth_bases(uint64_t seed, uint64_t i0, uint32_t n,
                                                     uint32_t* __restrict__ out) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fe<Fs> a = synth_scalar<Fs>(seed, i0 + i);
  if (fe_is_zero<Fs>(a)) a.l[0] = 1;
  const Aff<F> P = xyzz_to_aff<F>(scalar_mul<F, Fs>(a, generator<Cv>()));
  uint4* q = reinterpret_cast<uint4*>(out + 16ull * i);
  store_fe4<F>(q, P.x);
  store_fe4<F>(q + 2, P.y);
}

}  // namespace pm
