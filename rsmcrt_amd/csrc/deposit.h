// deposit.h — binned path-length deposition into jmean.
//
// The reference adds every voxel crossing straight into jmean with `!$omp atomic`
// (inttau2.f90:426-434). On MI355X a scattered device-scope atomic is a 64-B request at the
// memory side: ~22 G/s for the whole chip whatever its scope, type or locality (measured,
// profiles/r01_atomic_microbench.txt), and a wave cannot overlap them with its own
// compute. So the transport kernel instead appends 8-byte deposit records
// (voxel << 32 | f32 value) with wave-compacted stores into 128-KiB chunks of a record
// pool, and five small kernels fold them in:
//   bin_hist     records -> counts per (tile, bin block) (tile = TILE_VOXELS voxels)
//   bin_rowscan  counts  -> each bin block's offset inside each tile; tile totals
//   bin_scan     totals  -> tile offsets and the list of reduce pieces
//   bin_scatter  records -> tile-sorted order (LDS-staged, no global atomics)
//   bin_reduce   one piece of one tile per block: fp64 LDS accumulation, then the
//                tile's non-zero sums are added to the fp64 jmean
// Every record is read three times and written twice (40 B of HBM traffic per deposit,
// streamed and coalesced) instead of one scattered atomic.
// The value of a record is real(dcell,sp)*weight rounded to fp32, which is exact for the
// reference's unit-weight packets (noBiasPropagation); survival-bias runs use the atomic
// path so their fp64 weights are kept.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smcrt {

constexpr uint32_t CHUNK_RECORDS = 16384;  // 128 KiB per chunk
#ifndef SMCRT_TILE_SHIFT
#define SMCRT_TILE_SHIFT 14
#endif
constexpr uint32_t TILE_SHIFT = SMCRT_TILE_SHIFT;  // 16384 voxels per tile: 128 KiB of fp64 in LDS
constexpr uint32_t TILE_VOXELS = 1u << TILE_SHIFT;
constexpr uint32_t MAX_TILES = 4096;       // grids up to 2^26 voxels use the binned path
// A reduce piece is one block's share of one tile. Each piece ends with one fp64 atomic per
// touched voxel of its tile (up to TILE_VOXELS), so pieces are made as large as load balance
// allows: about REDUCE_PIECES pieces in total, and never smaller than MIN_PIECE_RECORDS.
constexpr uint32_t MIN_PIECE_RECORDS = 1u << 16;
constexpr uint32_t REDUCE_PIECES = 2048;

struct Piece {
  uint32_t tile, start, count, pad;
};

// Wave-uniform record-log cursor. Lives in scalar registers: it is only touched in
// wave-uniform control flow.
struct RecLog {
  uint32_t chunk;  // current chunk index (n_chunks: none yet / exhausted)
  uint32_t fill;   // records written into it
};

// Append one deposit per lane with dep == true. Must be called in wave-uniform control
// flow (every lane of the wave reaches it).
constexpr uint32_t LOG_NONE = 0xFFFFFFFFu;       // no chunk taken yet
constexpr uint32_t LOG_EXHAUSTED = 0xFFFFFFFEu;  // pool full: deposits fall back to atomics

__device__ __forceinline__ unsigned long long pack_record(uint32_t vox, double val) {
  return ((unsigned long long)vox << 32) | (unsigned long long)__float_as_uint((float)val);
}

#ifndef SMCRT_BIN_BLOCKS
#define SMCRT_BIN_BLOCKS 1024
#endif
constexpr uint32_t BIN_BLOCKS_ = SMCRT_BIN_BLOCKS;  // == BIN_BLOCKS below

// Add the wave's LDS tile histogram of chunk `chunk` into counts[tile][chunk % BIN_BLOCKS]
// and clear it (wave-uniform call; LDS ops of one wave complete in order).
__device__ __forceinline__ void flush_hist(const KParams& K, const KCold* __restrict__ C, uint32_t* whist,
                                           uint32_t chunk) {
  const int lane = threadIdx.x & 63;
  for (uint32_t t = lane; t < K.hist_tiles; t += 64) {
    const uint32_t v = whist[t];
    if (v) {
      atomicAdd(C->bin_counts + (uint64_t)t * BIN_BLOCKS_ + (chunk % BIN_BLOCKS_), v);
      whist[t] = 0;
    }
  }
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ void emit_deposits(const KParams& K, const KCold* __restrict__ C, RecLog& W, bool dep,
                                              uint32_t vox, double val, uint32_t& overflow, uint32_t* whist) {
  const uint64_t m = __ballot(dep);
  if (!m) return;
  // The cursor arithmetic is wave-uniform; readfirstlane keeps it (and the chunk address) on
  // the scalar unit, so a lane only pays for its rank, its store and its histogram add.
  const uint32_t n = (uint32_t)__popcll(m);
  const int lane = threadIdx.x & 63;
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  const bool fused = K.hist_tiles != 0;
  const unsigned long long rec = pack_record(vox, val);
  const uint32_t fill = uniform(W.fill);
  uint32_t chunk = uniform(W.chunk);
  uint32_t before = 0;  // lanes that still fit in the current chunk
  if (chunk < K.n_chunks) before = (CHUNK_RECORDS - fill) < n ? (CHUNK_RECORDS - fill) : n;
  if (before) {
    unsigned long long* const base = K.rec_pool + ((uint64_t)chunk * CHUNK_RECORDS + fill);
    if (dep && rank < before) {
      base[rank] = rec;
      if (fused) atomicAdd(whist + (vox >> TILE_SHIFT), 1u);
    }
  }
  W.fill = fill + before;
  W.chunk = chunk;
  if (before < n) {  // chunk full or none yet: retire it, take the next one
    const uint32_t rest = n - before;
    if (chunk != LOG_EXHAUSTED) {
      if (chunk < K.n_chunks && fused) flush_hist(K, C, whist, chunk);
      if (chunk < K.n_chunks && lane == 0) C->chunk_fill[chunk] = fill + before;
      uint32_t c = 0;
      if (lane == 0) c = atomicAdd(C->dep_ctl, 1u);
      c = uniform(c);  // lane 0 (every lane is active here)
      chunk = c < K.n_chunks ? c : LOG_EXHAUSTED;
    }
    if (chunk < K.n_chunks) {  // rest <= 64 < CHUNK_RECORDS
      unsigned long long* const base = K.rec_pool + (uint64_t)chunk * CHUNK_RECORDS;
      if (dep && rank >= before) {
        base[rank - before] = rec;
        if (fused) atomicAdd(whist + (vox >> TILE_SHIFT), 1u);
      }
      W.fill = rest;
    } else {  // pool exhausted: stay correct with fp64 atomics
      if (dep && rank >= before) atomic_add_nr(C->jmean + vox, val);
      overflow += rest;
      W.fill = 0;
    }
    W.chunk = chunk;
  }
}

__device__ __forceinline__ void close_log(const KParams& K, const KCold* __restrict__ C, RecLog& W,
                                          uint32_t overflow, uint32_t* whist) {
  const int lane = threadIdx.x & 63;
  if (W.chunk < K.n_chunks && K.hist_tiles) flush_hist(K, C, whist, W.chunk);
  if (lane == 0) {
    if (W.chunk < K.n_chunks) C->chunk_fill[W.chunk] = W.fill;
    if (overflow) atomicAdd(C->dep_ctl + 1, overflow);
  }
}

// Chunk c of the pool belongs to bin block c % BIN_BLOCKS in both bin_hist and bin_scatter,
// so every (tile, block) pair owns one contiguous run of the sorted array and the scatter
// needs no global atomics.
constexpr uint32_t BIN_BLOCKS = BIN_BLOCKS_;
constexpr int BIN_THREADS = 1024;
#ifndef SMCRT_STAGE_RECORDS
#define SMCRT_STAGE_RECORDS 8192
#endif
constexpr uint32_t STAGE_RECORDS = SMCRT_STAGE_RECORDS;        // records per LDS pass of bin_scatter
constexpr int STAGE_PER_THREAD = STAGE_RECORDS / BIN_THREADS;  // 8

__device__ __forceinline__ uint32_t rec_tile(unsigned long long x) { return (uint32_t)(x >> 32) >> TILE_SHIFT; }

// Exclusive scan of one value per thread over a 1024-thread block; *total gets the sum.
// `wsum` is 16 words of LDS. Ends with the block synchronised.
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) {
    const uint32_t t = wsum[i];
    before += i < w ? t : 0u;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

#ifdef SMCRT_FOLD_KERNELS  // (the fold kernels live in smcrt.hip's translation unit only)
// ---- bin_hist: record counts per (tile, bin block) -------------------------------------
__global__ __launch_bounds__(BIN_THREADS) void bin_hist(const unsigned long long* __restrict__ pool,
                                                        const uint32_t* __restrict__ chunk_fill,
                                                        const uint32_t* __restrict__ dep_ctl, uint32_t n_chunks,
                                                        uint32_t n_tiles, uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[MAX_TILES];
  for (uint32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) hist[t] = 0;
  __syncthreads();
  const uint32_t used = dep_ctl[0] < n_chunks ? dep_ctl[0] : n_chunks;
  for (uint32_t c = blockIdx.x; c < used; c += BIN_BLOCKS) {
    const uint32_t fill = chunk_fill[c];
    const unsigned long long* r = pool + (uint64_t)c * CHUNK_RECORDS;
    for (uint32_t i = threadIdx.x; i < fill; i += blockDim.x) atomicAdd(&hist[rec_tile(r[i])], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) counts[(uint64_t)t * BIN_BLOCKS + blockIdx.x] = hist[t];
}

// ---- bin_rowscan: per tile, exclusive scan over the bin blocks; tile totals ---------------
__global__ __launch_bounds__(BIN_BLOCKS) void bin_rowscan(uint32_t* __restrict__ counts,
                                                          uint32_t* __restrict__ tile_count) {
  __shared__ uint32_t wsum[16];
  uint32_t* row = counts + (uint64_t)blockIdx.x * BIN_BLOCKS;
  uint32_t total;
  const uint32_t ex = block_exscan(row[threadIdx.x], wsum, &total);
  row[threadIdx.x] = ex;
  if (threadIdx.x == 0) tile_count[blockIdx.x] = total;
}

// ---- bin_scan: tile offsets and reduce pieces (one block) ----------------------------------
__global__ __launch_bounds__(1024) void bin_scan(const uint32_t* __restrict__ tile_count, uint32_t n_tiles,
                                                 uint32_t* __restrict__ tile_start, Piece* __restrict__ pieces,
                                                 uint32_t* __restrict__ dep_ctl) {
  __shared__ uint32_t wsum[16];
  const uint32_t per = (n_tiles + blockDim.x - 1) / blockDim.x;
  const uint32_t t0 = threadIdx.x * per < n_tiles ? threadIdx.x * per : n_tiles;
  const uint32_t t1 = t0 + per < n_tiles ? t0 + per : n_tiles;
  uint32_t s = 0;
  for (uint32_t t = t0; t < t1; ++t) s += tile_count[t];
  uint32_t all_s, all_np;
  uint32_t off = block_exscan(s, wsum, &all_s);
  const uint32_t want = all_s / REDUCE_PIECES + 1;
  const uint32_t piece = want > MIN_PIECE_RECORDS ? want : MIN_PIECE_RECORDS;
  uint32_t np = 0;
  for (uint32_t t = t0; t < t1; ++t) np += (tile_count[t] + piece - 1) / piece;
  uint32_t pc = block_exscan(np, wsum, &all_np);
  if (threadIdx.x == 0) {
    dep_ctl[2] = all_np;  // number of pieces
    dep_ctl[3] = all_s;   // number of records
  }
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t c = tile_count[t];
    tile_start[t] = off;
    for (uint32_t k = 0; k < c; k += piece) {
      Piece p;
      p.tile = t; p.start = off + k; p.count = (c - k) < piece ? (c - k) : piece; p.pad = 0;
      pieces[pc++] = p;
    }
    off += c;
  }
}

// ---- bin_scatter: records into tile order --------------------------------------------------
// Block b walks the chunks c = b, b + BIN_BLOCKS, ... in passes of STAGE_RECORDS records:
//   A  rank: LDS atomic count per tile (the returned count is the record's rank)
//   B  wave 0: scan the counts -> off[t]; dest[t] = base[t] - off[t]; base[t] += count;
//      counts cleared for the next pass
//   C  place the records tile-ordered in LDS (stage[off[t] + rank])
//   D  write stage[j] to sorted[dest[t] + j]: consecutive threads, consecutive addresses
// The next pass's records are loaded during B-D. Three barriers per pass.
// Dynamic LDS: stage[STAGE_RECORDS] u64 | cnt[n_tiles] | off[n_tiles + 1] | dest[n_tiles] | base[n_tiles].
inline size_t scatter_lds_bytes(uint32_t n_tiles) {
  return STAGE_RECORDS * 8 + ((size_t)4 * n_tiles + 1) * 4;
}

__device__ __forceinline__ void load_stage(unsigned long long (&v)[STAGE_PER_THREAD],
                                           const unsigned long long* __restrict__ pool, uint32_t c, uint32_t h,
                                           uint32_t fill) {
  const unsigned long long* r = pool + (uint64_t)c * CHUNK_RECORDS + h;
  const uint32_t n = fill - h < STAGE_RECORDS ? fill - h : STAGE_RECORDS;
#pragma unroll
  for (int k = 0; k < STAGE_PER_THREAD; ++k) {
    const uint32_t i = threadIdx.x + k * BIN_THREADS;
    v[k] = i < n ? r[i] : 0ull;
  }
}

__global__ __launch_bounds__(BIN_THREADS) void bin_scatter(const unsigned long long* __restrict__ pool,
                                                           const uint32_t* __restrict__ chunk_fill,
                                                           const uint32_t* __restrict__ dep_ctl, uint32_t n_chunks,
                                                           uint32_t n_tiles, const uint32_t* __restrict__ tile_start,
                                                           const uint32_t* __restrict__ counts,
                                                           unsigned long long* __restrict__ sorted, uint64_t cap) {
  extern __shared__ unsigned long long stage[];
  uint32_t* cnt = (uint32_t*)(stage + STAGE_RECORDS);
  uint32_t* off = cnt + n_tiles;
  uint32_t* dest = off + n_tiles + 1;
  uint32_t* base = dest + n_tiles;
  const uint32_t used = dep_ctl[0] < n_chunks ? dep_ctl[0] : n_chunks;
  if (blockIdx.x >= used) return;  // block-uniform
  for (uint32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) {
    base[t] = tile_start[t] + counts[(uint64_t)t * BIN_BLOCKS + blockIdx.x];
    cnt[t] = 0;
  }
  const int lane = threadIdx.x & 63;
  const uint32_t per = (n_tiles + 63) / 64;  // wave-0 scan: consecutive tiles per lane
  const uint32_t t0 = lane * per < n_tiles ? lane * per : n_tiles;
  const uint32_t t1 = t0 + per < n_tiles ? t0 + per : n_tiles;

  uint32_t c = blockIdx.x, h = 0, fill = chunk_fill[c];
  unsigned long long v[STAGE_PER_THREAD];
  load_stage(v, pool, c, h, fill);
  __syncthreads();
  for (;;) {
    const uint32_t n = fill - h < STAGE_RECORDS ? fill - h : STAGE_RECORDS;
    uint32_t rank[STAGE_PER_THREAD];  // A
#pragma unroll
    for (int k = 0; k < STAGE_PER_THREAD; ++k) {
      const uint32_t i = threadIdx.x + k * BIN_THREADS;
      rank[k] = i < n ? atomicAdd(&cnt[rec_tile(v[k])], 1u) : 0u;
    }
    uint32_t cn = c, hn = h + STAGE_RECORDS, filln = fill;  // next pass, loaded during B-D
    if (hn >= fill) {
      cn = c + BIN_BLOCKS; hn = 0;
      filln = cn < used ? chunk_fill[cn] : 0u;
    }
    unsigned long long vn[STAGE_PER_THREAD];
    if (cn < used) load_stage(vn, pool, cn, hn, filln);
    __syncthreads();
    if (threadIdx.x < 64) {  // B
      uint32_t sum = 0;
      for (uint32_t t = t0; t < t1; ++t) sum += cnt[t];
      uint32_t x = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      uint32_t o = x - sum;
      for (uint32_t t = t0; t < t1; ++t) {
        const uint32_t k = cnt[t];
        off[t] = o;
        dest[t] = base[t] - o;
        base[t] += k;
        cnt[t] = 0;
        o += k;
      }
      if (lane == 63) off[n_tiles] = x;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < STAGE_PER_THREAD; ++k) {  // C
      const uint32_t i = threadIdx.x + k * BIN_THREADS;
      if (i < n) stage[off[rec_tile(v[k])] + rank[k]] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < STAGE_PER_THREAD; ++k) {  // D
      const uint32_t j = threadIdx.x + k * BIN_THREADS;
      if (j < n) {
        const unsigned long long x = stage[j];
        const uint64_t at = (uint64_t)dest[rec_tile(x)] + j;
        if (at < cap) sorted[at] = x;  // (guard: counts and records always agree)
      }
    }
    if (cn >= used) break;
    c = cn; h = hn; fill = filln;
#pragma unroll
    for (int k = 0; k < STAGE_PER_THREAD; ++k) v[k] = vn[k];
  }
}
#endif  // SMCRT_FOLD_KERNELS

// =============================================================================================
// Tile buckets: the transport kernel files each record straight into a bucket of its tile,
// so the fold reads every record once and writes nothing back (16 B of HBM traffic per
// deposit: the record's write and its read; the sorted path above moves 40 B).
//
// A bucket is BUCKET_RECORDS consecutive pool slots that hold records of one tile only.
// The four waves of a block share, in LDS, one 64-bit word per tile:
//   cur (24 bits) | next (24 bits) | fill (16 bits)
// `cur` is the tile's open bucket, `next` the bucket that follows it (taken in advance), and
// fill the records claimed in `cur`. A deposit is one LDS add-and-return of 1 on that word,
// which hands it its slot: fill < BUCKET_RECORDS -> cur[fill]; fill in [BUCKET_RECORDS,
// 2*BUCKET_RECORDS) -> next[fill - BUCKET_RECORDS], so no deposit waits for a claim in the
// common case. The deposit that found fill at exactly BUCKET_RECORDS takes the slow path: it
// makes `next` the open bucket, takes a fresh `next` from its wave's batch of ids
// (BUCKET_BATCH per returning atomic) and rebases fill with one compare-and-swap. A deposit
// that finds fill >= 2*BUCKET_RECORDS (both buckets full while that claim is still pending)
// places nothing: its lane waits until the claim has changed the word, then adds again.
//
// Why fill cannot carry into `next` (16 bits: 65536). fill only grows by deposit adds, and
// the claim's CAS is the only thing that lowers it. At most one claim per tile is pending:
// it is made by the one add that reads exactly BUCKET_RECORDS, and fill cannot read that
// value again before the CAS rebases it. While it is pending, the adds read BUCKET_RECORDS ..
// 2*BUCKET_RECORDS - 1 (each gets a slot in `next`) and then values >= 2*BUCKET_RECORDS; a
// lane whose add read such a value places nothing and adds again only after the word has
// changed (the CAS), so each of the block's 256 lanes makes at most one such add per pending
// claim. Hence fill <= 2*BUCKET_RECORDS + 256 = 768 however long the claiming wave takes
// (its returning batch atomic included), and the CAS caps it at 2*BUCKET_RECORDS before
// subtracting BUCKET_RECORDS. The claiming wave makes its claims before any of its own lanes
// wait, and a claim waits for nothing but its own atomics, so every wait ends.
// Sharing the words per block (round 2: per wave before) keeps 4x fewer buckets open, so
// their partly written cache lines fit in L2 and leave it whole.
// The fold (bk_scan, bk_place, bk_reduce) lists the buckets of each tile and sums them in LDS.
#ifndef SMCRT_REC6
#define SMCRT_REC6 1
#endif
// 6-byte records keep the voxel within the tile as a u16
static_assert(!SMCRT_REC6 || TILE_SHIFT <= 16, "SMCRT_REC6 records need tiles of at most 2^16 voxels");
constexpr uint32_t BUCKET_SHIFT = 8;
constexpr uint32_t BUCKET_RECORDS = 1u << BUCKET_SHIFT;  // 2 KiB per bucket
#ifndef SMCRT_BUCKET_BATCH
#define SMCRT_BUCKET_BATCH 64
#endif
constexpr uint32_t BUCKET_BATCH = SMCRT_BUCKET_BATCH;    // ids a wave takes at a time
// One deposit wave-instruction makes at most 64 claims (one per lane) and the batch must
// cover them (bucket_slow takes at most one new batch per instruction); the retirement of
// unused ids (one lane per id) covers at most 64 ids. Both hold exactly for 64.
static_assert(BUCKET_BATCH == 64, "bucket id batches must be exactly one id per lane of a wave");
constexpr uint32_t BUCKET_ID_NONE = 0xFFFFFFu;           // no bucket (24-bit id field)
constexpr uint32_t BUCKET_ID_EXHAUSTED = 0xFFFFFEu;      // pool full: the tile's deposits use atomics
constexpr uint32_t TILE_INVALID = 0xFFFFFFFFu;           // bucket_tile of an id never used
constexpr uint32_t MAX_DIRECT_TILES = 1024;              // 8 B of LDS per tile per block
constexpr uint32_t MIN_PIECE_BUCKETS = MIN_PIECE_RECORDS / BUCKET_RECORDS;
// (pool ids stay below 2^24 - 2^20: MAX_POOL_RECORDS <= 2^32 - 2^28 records)

// Wave-uniform batch of bucket ids [next, end) (scalar registers).
struct BucketLog {
  uint32_t next, end;
};

__device__ __forceinline__ unsigned long long bucket_word(uint32_t cur, uint32_t next, uint32_t fill) {
  return ((unsigned long long)cur << 40) | ((unsigned long long)next << 16) | fill;
}
__device__ __forceinline__ uint32_t bw_cur(unsigned long long w) { return (uint32_t)(w >> 40); }
__device__ __forceinline__ uint32_t bw_next(unsigned long long w) { return (uint32_t)(w >> 16) & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t bw_fill(unsigned long long w) { return (uint32_t)w & 0xFFFFu; }

// Block start (every thread calls it; the caller's barrier publishes the words): one id per
// tile taken as the tiles' first `next`; fill = BUCKET_RECORDS makes the first deposit of a
// tile open it.
__device__ __forceinline__ void init_buckets(const KParams& K, const KCold* __restrict__ C, unsigned long long* bs) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(C->dep_ctl, K.bucket_tiles);
  base = uniform(__shfl(base, 0, 64));
  for (uint32_t t = lane; t < K.bucket_tiles; t += 64) {
    const uint32_t id = base + t;
    bs[t] = bucket_word(BUCKET_ID_NONE, id < K.n_buckets ? id : BUCKET_ID_EXHAUSTED, BUCKET_RECORDS);
  }
}

// The rare part of a deposit instruction (wave-uniform call): the claims of the lanes that
// found fill == BUCKET_RECORDS, and the exact atomic for lanes whose bucket does not exist
// (pool exhausted).
__device__ __forceinline__ void bucket_slow(const KParams& K, const KCold* __restrict__ C, BucketLog& W,
                                            bool claim, bool spill, unsigned long long w, uint32_t t,
                                            uint32_t vox, double val, uint32_t& overflow, unsigned long long* bs) {
  const int lane = threadIdx.x & 63;
  const uint64_t cm = __ballot(claim);
  const uint32_t nc = (uint32_t)__popcll(cm);
  uint32_t next = uniform(W.next), end = uniform(W.end);
  if (nc > end - next) {  // batch used up: retire its unused ids, take a new batch
    const uint32_t id = next + lane;
    if (id < end && id < K.n_buckets) C->bucket_tile[id] = TILE_INVALID;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(C->dep_ctl, BUCKET_BATCH);
    base = uniform(__shfl(base, 0, 64));
    next = base;
    end = base + BUCKET_BATCH;
  }
  if (claim) {
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
    const uint32_t fresh = next + rank < K.n_buckets ? next + rank : BUCKET_ID_EXHAUSTED;
    const uint32_t cur = bw_cur(w), nx = bw_next(w);
    if (cur < K.n_buckets) C->bucket_fill[cur] = BUCKET_RECORDS;  // the full bucket
    if (nx < K.n_buckets) {  // `next` becomes the tile's open bucket
      C->bucket_tile[nx] = t;
      atomicAdd(C->tile_nb + t, 1u);
    }
    // debug knob (SMCRT_DEBUG_CLAIM_DELAY, tests only): hold the claim open so that other
    // waves fill both buckets and wait
    for (uint32_t d = 0; d < K.claim_delay; ++d) __builtin_amdgcn_s_sleep(127);
    // cur <- next, next <- fresh, fill -= BUCKET_RECORDS; adds that found fill >=
    // 2*BUCKET_RECORDS placed nothing (their lanes add again after this), so fill is capped
    // first and the deposit that finds BUCKET_RECORDS again opens `fresh`. Only this lane
    // changes cur/next while its claim is pending, so they are still (cur, nx) here.
    unsigned long long old = __hip_atomic_load(bs + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
      const uint32_t f = bw_fill(old);
      const uint32_t f2 = (f < 2 * BUCKET_RECORDS ? f : 2 * BUCKET_RECORDS) - BUCKET_RECORDS;
      const unsigned long long nw = bucket_word(nx, fresh, f2);
      if (__hip_atomic_compare_exchange_strong(bs + t, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP))
        break;
    }
  }
  W.next = next + nc;
  W.end = end;
  if (spill) atomic_add_nr(C->jmean + vox, val);  // exact fp64 fallback
  overflow += (uint32_t)__popcll(__ballot(spill));
}

// File one deposit per lane with dep == true (wave-uniform call).
__device__ __forceinline__ void emit_bucketed(const KParams& K, const KCold* __restrict__ C, BucketLog& W, bool dep,
                                              uint32_t vox, double val, uint32_t& overflow,
                                              unsigned long long* bs) {
  if (!__ballot(dep)) return;
  const uint32_t t = vox >> TILE_SHIFT;
  bool todo = dep;
  for (;;) {  // wave-uniform; one pass unless a lane found both of its tile's buckets full
    unsigned long long w = 0;
    if (todo) w = __hip_atomic_fetch_add(bs + t, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t pos = bw_fill(w);
    const uint32_t b = pos < BUCKET_RECORDS ? bw_cur(w) : bw_next(w);
    const bool slot = todo && pos < 2 * BUCKET_RECORDS;
    const bool ok = slot && b < K.n_buckets;
    if (ok) {
#if SMCRT_REC6
      // 6-byte records (round 5): the bucket's tile is implied, so a record is its f32 value
      // (first KiB of the bucket) and its 14-bit voxel within the tile (the next 512 B)
      uint32_t* const bv = (uint32_t*)(K.rec_pool + ((uint64_t)b << BUCKET_SHIFT));
      const uint32_t slot = pos & (BUCKET_RECORDS - 1);
      bv[slot] = __float_as_uint((float)val);
      ((uint16_t*)(bv + BUCKET_RECORDS))[slot] = (uint16_t)(vox & (TILE_VOXELS - 1));
#else
      K.rec_pool[((uint64_t)b << BUCKET_SHIFT) + (pos & (BUCKET_RECORDS - 1))] = pack_record(vox, val);
#endif
    }
    const bool claim = todo && pos == BUCKET_RECORDS;
    const bool spill = slot && !ok;
    const bool wait = todo && !slot;  // both buckets full: a claim is pending in another wave
    if (!__ballot(claim || spill || wait)) return;
    bucket_slow(K, C, W, claim, spill, w, t, vox, val, overflow, bs);
    if (!__ballot(wait)) return;
    bool expired = false;
    if (wait) {  // until the pending claim has rebased the word (see the bound above)
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      unsigned long long x;
      do {
        __builtin_amdgcn_s_sleep(2);
        x = __hip_atomic_load(bs + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // (the watchdog: a claim that never lands drops this record and fails the run)
        if (watchdog_expired(C, t0, WDOG_BUCKET)) { expired = true; break; }
      } while (bw_fill(x) >= 2 * BUCKET_RECORDS && bw_cur(x) == bw_cur(w));
    }
    todo = wait && !expired;
  }
}

// End of the kernel for one wave: retire the unused ids of its batch and add its record and
// overflow counts. (close_block_buckets then closes the block's words.)
__device__ __forceinline__ void close_buckets(const KParams& K, const KCold* __restrict__ C, const BucketLog& W,
                                              uint32_t records, uint32_t overflow) {
  const int lane = threadIdx.x & 63;
  const uint32_t id = W.next + lane;
  if (id < W.end && id < K.n_buckets) C->bucket_tile[id] = TILE_INVALID;
  if (lane == 0) {
    if (records) atomicAdd(C->dep_ctl + 3, records);
    if (overflow) atomicAdd(C->dep_ctl + 1, overflow);
  }
}
// After the block's last deposit (behind a block barrier; every thread calls it): the fill of
// each open bucket, and the unused `next` ids retired. No claim is pending here, so fill is
// at most BUCKET_RECORDS and nothing was written into `next`.
__device__ __forceinline__ void close_block_buckets(const KParams& K, const KCold* __restrict__ C,
                                                    const unsigned long long* bs) {
  for (uint32_t t = threadIdx.x; t < K.bucket_tiles; t += blockDim.x) {
    const unsigned long long w = bs[t];
    const uint32_t cur = bw_cur(w), nx = bw_next(w), f = bw_fill(w);
    if (cur < K.n_buckets) C->bucket_fill[cur] = f < BUCKET_RECORDS ? f : BUCKET_RECORDS;
    if (nx < K.n_buckets) C->bucket_tile[nx] = TILE_INVALID;
  }
}

#ifdef SMCRT_FOLD_KERNELS
// ---- bk_scan: bucket offsets per tile and the reduce pieces (one block) --------------------
// tile_nb[t] buckets of tile t -> tile_start[t] (exclusive scan), cursor[t] = tile_start[t];
// pieces of at most `pb` buckets of one tile. dep_ctl[2] = pieces.
__global__ __launch_bounds__(1024) void bk_scan(const uint32_t* __restrict__ tile_nb, uint32_t n_tiles,
                                                uint32_t* __restrict__ tile_start, uint32_t* __restrict__ cursor,
                                                Piece* __restrict__ pieces, uint32_t* __restrict__ dep_ctl) {
  __shared__ uint32_t wsum[16];
  const uint32_t per = (n_tiles + blockDim.x - 1) / blockDim.x;
  const uint32_t t0 = threadIdx.x * per < n_tiles ? threadIdx.x * per : n_tiles;
  const uint32_t t1 = t0 + per < n_tiles ? t0 + per : n_tiles;
  uint32_t s = 0;
  for (uint32_t t = t0; t < t1; ++t) s += tile_nb[t];
  uint32_t all_s, all_np;
  uint32_t off = block_exscan(s, wsum, &all_s);
  const uint32_t want = all_s / REDUCE_PIECES + 1;
  const uint32_t pb = want > MIN_PIECE_BUCKETS ? want : MIN_PIECE_BUCKETS;
  uint32_t np = 0;
  for (uint32_t t = t0; t < t1; ++t) np += (tile_nb[t] + pb - 1) / pb;
  uint32_t pc = block_exscan(np, wsum, &all_np);
  if (threadIdx.x == 0) dep_ctl[2] = all_np;
  for (uint32_t t = t0; t < t1; ++t) {
    const uint32_t c = tile_nb[t];
    tile_start[t] = off;
    cursor[t] = off;
    for (uint32_t k = 0; k < c; k += pb) {
      Piece p;
      p.tile = t; p.start = off + k; p.count = (c - k) < pb ? (c - k) : pb; p.pad = 0;
      pieces[pc++] = p;
    }
    off += c;
  }
}

// ---- bk_place: bucket ids in tile order ------------------------------------------------------
// Block b takes a contiguous range of ids in passes of BIN_THREADS * 8: LDS ranks per tile,
// one global reservation per (pass, tile), then the ids are written to order[].
__global__ __launch_bounds__(BIN_THREADS) void bk_place(const uint32_t* __restrict__ bucket_tile,
                                                        const uint32_t* __restrict__ dep_ctl, uint32_t n_buckets,
                                                        uint32_t n_tiles, uint32_t* __restrict__ cursor,
                                                        uint32_t* __restrict__ order) {
  __shared__ uint32_t cnt[MAX_DIRECT_TILES];
  __shared__ uint32_t base[MAX_DIRECT_TILES];
  const uint32_t used = dep_ctl[0] < n_buckets ? dep_ctl[0] : n_buckets;
  const uint32_t per = (used + gridDim.x - 1) / gridDim.x;
  const uint32_t b0 = blockIdx.x * per;
  const uint32_t b1 = b0 + per < used ? b0 + per : used;
  constexpr int PER_THREAD = 8;
  for (uint32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) cnt[t] = 0;
  __syncthreads();
  for (uint32_t p = b0; p < b1; p += BIN_THREADS * PER_THREAD) {
    uint32_t tile[PER_THREAD], rank[PER_THREAD];
#pragma unroll
    for (int k = 0; k < PER_THREAD; ++k) {
      const uint32_t i = p + threadIdx.x + k * BIN_THREADS;
      tile[k] = i < b1 ? bucket_tile[i] : TILE_INVALID;
      rank[k] = tile[k] < n_tiles ? atomicAdd(&cnt[tile[k]], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n_tiles; t += blockDim.x) {
      const uint32_t c = cnt[t];
      base[t] = c ? atomicAdd(cursor + t, c) : 0u;
      cnt[t] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER_THREAD; ++k) {
      const uint32_t i = p + threadIdx.x + k * BIN_THREADS;
      if (tile[k] < n_tiles) order[base[tile[k]] + rank[k]] = i;
    }
    __syncthreads();
  }
}

// ---- bk_reduce: one piece (buckets of one tile) per block, fp64 LDS sums into jmean --------
// (blockDim.x must be 1024)
constexpr uint32_t RED_THREADS = 1024;  // bk_reduce's block size
// One wave per bucket (round 4): wave w of the block takes buckets w, w + 16, w + 32, ... of the
// piece, RED_GROUP at a time; a bucket's id and fill are scalar loads and its 256 records four
// coalesced 512-B loads per wave. The next group's records are loaded before this group's LDS
// adds are issued (software pipeline), so each wave keeps 2 * RED_GROUP * 4 records per lane
// in flight and its memory latency overlaps its own LDS atomics; no ids/fills staging in LDS
// and no block barrier inside a piece. Sums are the same fp64 LDS adds in a different order.
// (Measured and removed in round 5: a block-wide staged variant with 16 loads in flight per
// thread, 5 % slower; non-temporal record loads, no change, profiles/r03_s3/nt_ab.txt.)
constexpr int RED_GROUP = 4;
__global__ __launch_bounds__(RED_THREADS) void bk_reduce(const unsigned long long* __restrict__ pool,
                                                  const uint32_t* __restrict__ order,
                                                  const uint32_t* __restrict__ bucket_fill,
                                                  const Piece* __restrict__ pieces,
                                                  const uint32_t* __restrict__ dep_ctl, uint64_t n_voxels,
                                                  double* __restrict__ jmean, unsigned long long* __restrict__ busy) {
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  __shared__ double acc[TILE_VOXELS];
  const uint32_t n_pieces = dep_ctl[2];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr uint32_t NW = RED_THREADS / 64;  // waves per block
  constexpr int NR = RED_GROUP * 4;        // records per lane per group
  for (uint32_t pi = blockIdx.x; pi < n_pieces; pi += gridDim.x) {
    const Piece p = pieces[pi];
    for (uint32_t i = threadIdx.x; i < TILE_VOXELS; i += blockDim.x) acc[i] = 0.0;
    __syncthreads();
    // group g of this wave: buckets w + NW * (RED_GROUP * g + u), u < RED_GROUP
    auto fetch = [&](uint32_t g, unsigned long long* x) {
#pragma unroll
      for (int u = 0; u < RED_GROUP; ++u) {
        const uint32_t b = w + NW * (RED_GROUP * g + (uint32_t)u);
        uint32_t f = 0, id = 0;
        if (b < p.count) {
          id = uniform(order[p.start + b]);
          f = uniform(bucket_fill[id]);
        }
        const unsigned long long* __restrict__ base = pool + ((uint64_t)id << BUCKET_SHIFT);
#if SMCRT_REC6
        const uint32_t* __restrict__ bv = (const uint32_t*)base;
        const uint16_t* __restrict__ bi = (const uint16_t*)(bv + BUCKET_RECORDS);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t slot = lane + 64u * (uint32_t)r;
          x[4 * u + r] = slot < f ? ((unsigned long long)bi[slot] << 32) | bv[slot] : ~0ull;
        }
#else
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t slot = lane + 64u * (uint32_t)r;
          x[4 * u + r] = slot < f ? base[slot] : ~0ull;
        }
#endif
      }
    };
    const uint32_t ng = (p.count + NW * RED_GROUP - 1) / (NW * RED_GROUP);  // groups of the piece (wave 0's count)
    unsigned long long cur[NR];
    fetch(0, cur);
    for (uint32_t g = 0; g < ng; ++g) {
      unsigned long long nxt[NR];
      if (g + 1 < ng) fetch(g + 1, nxt);
#pragma unroll
      for (int k = 0; k < NR; ++k)
        if (cur[k] != ~0ull) atomicAdd(&acc[(uint32_t)(cur[k] >> 32) & (TILE_VOXELS - 1)], (double)__uint_as_float((uint32_t)cur[k]));
      if (g + 1 < ng) {
#pragma unroll
        for (int k = 0; k < NR; ++k) cur[k] = nxt[k];
      }
    }
    __syncthreads();
    const uint64_t base = (uint64_t)p.tile << TILE_SHIFT;
    for (uint32_t i = threadIdx.x; i < TILE_VOXELS; i += blockDim.x) {
      const double a = acc[i];
      if (a != 0.0 && base + i < n_voxels) atomic_add_nr(jmean + base + i, a);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && busy) atomicAdd(busy, __builtin_amdgcn_s_memrealtime() - t_start);
}

// ---- bin_reduce: one tile piece per block, fp64 LDS sums added into jmean ----------------
// (blockDim.x must be 1024)
__global__ __launch_bounds__(1024) void bin_reduce(const unsigned long long* __restrict__ sorted,
                                                   const Piece* __restrict__ pieces,
                                                   const uint32_t* __restrict__ dep_ctl, uint64_t n_voxels,
                                                   double* __restrict__ jmean) {
  __shared__ double acc[TILE_VOXELS];
  const uint32_t n_pieces = dep_ctl[2];
  for (uint32_t pi = blockIdx.x; pi < n_pieces; pi += gridDim.x) {
    const Piece p = pieces[pi];
    for (uint32_t i = threadIdx.x; i < TILE_VOXELS; i += blockDim.x) acc[i] = 0.0;
    __syncthreads();
    const unsigned long long* r = sorted + p.start;
    uint32_t i = threadIdx.x;
    for (; i + 7 * 1024 < p.count; i += 8 * 1024) {  // 8 loads in flight per thread
      unsigned long long x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = r[i + k * 1024];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        atomicAdd(&acc[(uint32_t)(x[k] >> 32) & (TILE_VOXELS - 1)], (double)__uint_as_float((uint32_t)x[k]));
    }
    for (; i < p.count; i += 1024) {
      const unsigned long long x = r[i];
      atomicAdd(&acc[(uint32_t)(x >> 32) & (TILE_VOXELS - 1)], (double)__uint_as_float((uint32_t)x));
    }
    __syncthreads();
    const uint64_t base = (uint64_t)p.tile << TILE_SHIFT;
    for (uint32_t i = threadIdx.x; i < TILE_VOXELS; i += blockDim.x) {
      const double a = acc[i];
      if (a != 0.0 && base + i < n_voxels) atomic_add_nr(jmean + base + i, a);
    }
    __syncthreads();
  }
}
#endif  // SMCRT_FOLD_KERNELS

}  // namespace smcrt
