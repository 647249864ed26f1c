// mph_kernels.hip -- hand-written HIP/CDNA4 (gfx950) kernels of the MPH explicit hot path.
//
// One time step of the reference (main.cpp:597-686) is mapped onto these launches:
//
//   k_prep           calculateWall (3031-3071) + calculatePeriodicBoundary (3322-3333) + cell key
//                    + cell histogram (first half of the counting sort that replaces the
//                    reference's bitonic sort, 1683-1708)
//   k_scan_*         exclusive scan of the cell histogram -> cell start offsets (1711-1728)
//   k_place          scatter particle ids into their cells (unordered) + Time/WallCenter advance
//   k_rank_scatter   deterministic in-cell rank (by previous sorted index) and particle reorder
//   k_neighbors      linked-cell search (1743-1810): 7x7(x5) stencil (2 kReach + 1 columns of cells
//                    >= rc/3, 2 kContigReach + 1 cells >= rc/2 along the contiguous axis), the
//                    reference's exact FP64 acceptance test, ELL neighbour list per wavefront
//   k_pass_a         the pass-A sums over the list: DensityA (2141), GravityCenter (2174), DensityP
//                    (2314), DivergenceP (2343), PhysicalCoefficients (2099), pressure values
//                    PressureP (2384) / PressureA (2218)
//   k_pass_b         PressureP force (2394), PressureA force (2225), DiffuseInterface (2261),
//                    ViscosityV (2478), InterfaceForce (2427), Gravity (2917), Acceleration (2938),
//                    Convection (1892)
//   k_struct_*       elastic substeps: DeformationVector (2673) + Stress (2756) -> PK1 stress;
//                    StressForce (2812) in gather form + updateElasticPosition (1910); pass B
//                    hands the structure particles to them and the last substep writes back
//
// All arithmetic is FP64.  Neighbour membership and every per-kernel radius test reproduce the
// reference's FP64 expressions bit for bit (no contraction, IEEE division), so NeighborCount is
// exact; the weighted sums are reassociated (own order, FMA) and agree within the tolerances
// written in tests/.
//
// Memory layout: particle state is structure-of-arrays FP64 in cell-sorted order (Soa).  The
// neighbour loops are bound by the per-CU texture-address path (profiles/r01: TA ~75% busy with
// 32-byte records); SoA makes consecutive lanes gather consecutive doubles.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <climits>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "mph_kernels.h"
#include "mph_params.h"

// Tuning parameters (A/B builds: tools/ab.sh).  The rejected variants of rounds 1-5 (staged pass A,
// row spreading, CU-affine tiles, paired / half-wave / compact 16-bit lists, chunked search, cache-
// policy hints, record planes for pass A, block totals from k_prep, the diagnostic builds) were
// removed in round 6; they are kept under the git tag r05-variants (profiles/r05/README.md).
#ifndef MPH_SB
// candidates per batch in the search: 2 (64 VGPRs) with the LDS capacity below gives 8 waves per
// SIMD (round 3: D1M 0.355 -> 0.347 ms, D16M 4.11 -> 3.86, profiles/r03/search/sb2/); 3 took
// 72 VGPRs and 7 waves (round 2: 0.395 ms against 0.433 at 4)
#define MPH_SB 2
#endif
#ifndef MPH_LDS_CAP
// staging area per wave and stencil column, in FP64 candidates: 176 keeps a wave's staging at
// 5,072 B, so 32 waves (8 per SIMD) fit the 160 KB of LDS; it holds 313 of the 16-byte FP32
// records (kCap32), wider windows take the global-gather loop
#define MPH_LDS_CAP 176
#endif

namespace mph {

// Buffer descriptor of a device array (gfx9 raw-buffer format word, 4 GiB of records): loads through
// it take a 32-bit unsigned byte offset from a VGPR instead of a 64-bit address.  The cell table
// (ncell + 1 ints, checked at creation) and the particle arrays (< 2^28 entries) stay below 4 GiB.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t arr_rsrc(const void* p)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, -1, 0x00020000);
}
// a buffer descriptor over `bytes` bytes: loads past them return zeros without a memory access
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sized_rsrc(const void* p, unsigned bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
// 16 bytes at byte offset off of a buffer, as two doubles
__device__ __forceinline__ double2 buf_ld16(__amdgpu_buffer_rsrc_t r, unsigned off)
{
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return __builtin_bit_cast(double2, v);
}
__device__ __forceinline__ __attribute__((address_space(3))) void* lds_ptr(void* p)
{
    return (__attribute__((address_space(3))) void*)p;
}

// A 4-byte load through a buffer descriptor that hipcc does not count (the search's start[]
// loads, scan_candidates_lds): no s_waitcnt is emitted for it, so the caller waits for it with an
// explicit vmcnt(0) on every path before start_landed() and the first use of the value.
// Both bounds of a column range in one statement: the descriptor may come from SGPRs that a VALU
// instruction (v_readlane of an SGPR spill) has just written, which a VMEM instruction may read only
// 5 wait states later (hipcc pads only what it sees: s_nop 4 opens the string).
__device__ __forceinline__ void start_load2(__amdgpu_buffer_rsrc_t r, unsigned ob, unsigned oe, int& b, int& e)
{
    asm volatile("s_nop 4\n\tbuffer_load_dword %0, %2, %4, 0 offen\n\tbuffer_load_dword %1, %3, %4, 0 offen"
                 : "=&v"(b), "=&v"(e) : "v"(ob), "v"(oe), "s"(r) : "memory");
}
// marks the start_load2 results as landed: no consumer is scheduled above this point
__device__ __forceinline__ void start_landed(int& a, int& b) { asm volatile("" : "+v"(a), "+v"(b)); }

// LDS staging area of one wavefront in the search, in doubles: sized as the FP64 staging of CAP
// candidates (x, y, z: stage_d doubles each, types: stage_t ints) of rounds 1-4, which it holds the
// FP32 records of (16 bytes each, scan_candidates_lds kCap32).
__host__ __device__ constexpr int stage_d(int cap, int sb) { return (cap + sb + 2 + 1) & ~1; }
__host__ __device__ constexpr int stage_t(int cap, int sb) { return (cap + sb + 8 + 3) & ~3; }
__host__ __device__ constexpr int stage_words(int cap, int sb) { return 3 * stage_d(cap, sb) + stage_t(cap, sb) / 2; }


// ------------------------------------------------------------------------------ helpers ------

// Mod(x,w) of main.cpp:98, exact (IEEE division, floor, no contraction).
__device__ __forceinline__ double mod_exact(double x, double w)
{
#pragma clang fp contract(off)
    return x - w * floor(x / w);
}

// Periodic minimum image Mod(d + w/2, w) - w/2 of every pair loop (e.g. main.cpp:1762), bit-
// identical to the reference.  For 0 <= s < 0.75 w, floor(s/w) == 0 exactly and
// Mod(s,w) == s - w*0 == s; FAST (wave-uniform, interior particles only) relies on that always.
template <bool FAST>
__device__ __forceinline__ double image_exact(double d, double w, double hw, double w075)
{
#pragma clang fp contract(off)
    const double s = d + hw;
    double m;
    if (FAST || __builtin_expect(s >= 0.0 && s < w075, 1)) {
        m = s;
    } else {
        m = s - w * floor(s / w);
    }
    return m - hw;
}

__device__ __forceinline__ double r2_exact(double q0, double q1, double q2)
{
#pragma clang fp contract(off)
    return q0 * q0 + q1 * q1 + q2 * q2;
}

// r = sqrt(r2) and 1/r from v_rsq_f64 plus one Newton step (relative error ~1e-16).
__device__ __forceinline__ void rsqrt_pair(double r2, double& r, double& ir)
{
    double y = __builtin_amdgcn_rsq(r2);
    const double e = fma(-(r2 * y), y, 1.0);
    y = fma(0.5 * y, e, y);
    ir = y;
    r = r2 * y;
}

__device__ __forceinline__ int wrap_cell(int c, int g)
{
    c = c < 0 ? c + g : c;
    return c >= g ? c - g : c;
}

// Cell index along one axis.  The offset from the grid origin is wrapped once into [0, w) (w =
// periodic domain width), so a slab window that straddles the periodic seam (multi-GPU) sees its
// ghosts from the far side at the right place; for the full-domain grid the wrap changes nothing.
// Out-of-window offsets clamp into the edge cells (only far ghosts, never needed as neighbours).
__device__ __forceinline__ int cell_axis(double x, double org, double w, double ginv, int g)
{
    double u = x - org;
    u = u < 0.0 ? u + w : (u >= w ? u - w : u);
    // clamp before the conversion: a NaN / infinite coordinate (diverged input) maps to cell 0
    // instead of an undefined float->int conversion
    const double t = fmin(fmax(floor(u * ginv), 0.0), (double)(g - 1));
    return (int)t;
}

// linear cell index in the cell order DevParams.perm (order_axis; the last axis contiguous, with
// half-width cells)
__device__ __forceinline__ int cell_index(const DevParams& P, int cx, int cy, int cz)
{
    const int* g = P.gc;
    switch (P.perm) {
    case 1: return (cz * g[0] + cx) * g[1] + cy;   // (z, x, y)
    case 2: return (cz * g[1] + cy) * g[0] + cx;   // (z, y, x)
    case 3: return (cy * g[2] + cz) * g[0] + cx;   // (y, z, x)
    case 4: return (cx * g[2] + cz) * g[1] + cy;   // (x, z, y)
    default: return (cx * g[1] + cy) * g[2] + cz;  // (x, y, z)
    }
}

__device__ __forceinline__ int cell_id(const DevParams& P, double x, double y, double z)
{
    const int cx = cell_axis(x, P.corg[0], P.dw[0], P.ginv[0], P.gc[0]);
    const int cy = cell_axis(y, P.corg[1], P.dw[1], P.ginv[1], P.gc[1]);
    const int cz = P.dim == 3 ? cell_axis(z, P.corg[2], P.dw[2], P.ginv[2], P.gc[2]) : 0;
    return cell_index(P, cx, cy, cz);
}

// Logical axes of the cell order for the search: the two column axes (A0 slowest, A1) and the
// contiguous axis A2 (cells half as wide); 2-D: x columns, y contiguous.
template <int DIM, int PERM> struct CellAxes {
    static constexpr int A0 = DIM == 3 ? order_axis(PERM, 0) : 0;
    static constexpr int A1 = DIM == 3 ? order_axis(PERM, 1) : 1;
    static constexpr int A2 = DIM == 3 ? order_axis(PERM, 2) : 1;
};

__device__ __forceinline__ bool dev_is_struct(int t) { return t == 2 || t == 3; }
__device__ __forceinline__ bool dev_is_fluid(int t) { return t == 0 || t == 1; }
__device__ __forceinline__ bool dev_is_wall(int t) { return t == 4 || t == 5; }

// wave-uniform: every live lane's particle is >= 3 GPU cells away from every periodic face,
// so no stencil cell wraps and every candidate's minimum image takes the fast path.
__device__ __forceinline__ bool wave_interior(const DevParams& P, bool live, double x, double y, double z)
{
    bool in = !live || (x >= P.inner_lo[0] && x <= P.inner_hi[0] && y >= P.inner_lo[1] &&
                        y <= P.inner_hi[1] && (P.dim == 2 || (z >= P.inner_lo[2] && z <= P.inner_hi[2])));
    return P.fast_ok && __all(in);
}

// Particles of this lane within the face box margin of a periodic face: bit 2k low face, 2k + 1
// high face of axis k (k_prep gathers them per step into DevState.seam_occ).
__device__ __forceinline__ int seam_bits(const DevParams& P, double x, double y, double z)
{
    const double v[3] = {x, y, z};
    int b = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (k == 2 && P.dim == 2) break;
        if ((P.seam_always >> k) & 1) continue;   // (the slab axis: the face box always applies)
        b |= (v[k] < P.inner_lo[k] ? 1 : 0) << (2 * k);
        b |= (v[k] > P.inner_hi[k] ? 2 : 0) << (2 * k);
    }
    return b;
}

// wave-uniform, for the search: every live lane is >= 3 cells inside the cell grid's faces (so no
// stencil row wraps) and, on every axis with particles near BOTH periodic faces (this step's
// seam_occ) or on the slab axis, also >= 3 cells from the domain's faces (so no candidate pair
// straddles the periodic seam and the raw differences are the minimum image).  With the grid
// origin at dmin this is wave_interior; with the origin in an empty band it also admits the waves
// at a wall on a periodic face whose far side is empty (the dam's bottom wall).
__device__ __forceinline__ bool wave_search_interior(const DevParams& P, const DevState* st, bool live,
                                                     double x, double y, double z)
{
    const int occ = st->seam_occ[(st->seam_step - 1) & 1];
    const double v[3] = {x, y, z};
    bool in = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (k == 2 && P.dim == 2) break;
        double u = v[k] - P.corg[k];
        u = u < 0.0 ? u + P.dw[k] : (u >= P.dw[k] ? u - P.dw[k] : u);
        in = in && u >= P.sinner_lo[k] && u <= P.sinner_hi[k];
        const bool seam = ((P.seam_always >> k) & 1) || ((occ >> (2 * k)) & 3) == 3;
        if (seam) in = in && v[k] >= P.inner_lo[k] && v[k] <= P.inner_hi[k];
    }
    return P.fast_ok && __all(!live || in);
}

// XCD-aware block order: hardware deals consecutive blocks round-robin over the 8 XCDs; remap so
// that each XCD sweeps one contiguous 1/8 of the (cell-sorted) particles and neighbour gathers
// hit its own L2 (cdna_hip_programming.md T1, bijective form).
__device__ __forceinline__ int xcd_block(int b, int nb)
{
    const int xcd = b & 7;
    const int q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// Particles held by this context: exact on a single GPU; in slab mode the device-resident count
// of the last redistribution (P.n is then only the capacity the grids are sized for).
__device__ __forceinline__ int dev_n(const DevParams& P) { return P.n_dev ? *P.n_dev : P.n; }

// Blocks of 256 that hold live particles; the rest of a capacity-sized grid exits at once.  The
// XCD remap runs over the live blocks only, so the work stays spread over all 8 XCDs.
__device__ __forceinline__ int live_blocks(int n) { return (n + 255) >> 8; }

// Threads per block of the three list kernels (search, pass A, pass B): MPH_LB / 64 wavefronts
#ifndef MPH_LB
#define MPH_LB 256
#endif
constexpr int kWB = MPH_LB / 64;
__device__ __forceinline__ int list_blocks(int n) { return (n + MPH_LB - 1) / MPH_LB; }

// Work-balanced XCD map of the two list passes.  The waves' work is not uniform along the sorted
// order (walls, the free surface, a slab's ghost waves), so equal block counts per XCD leave some
// XCDs idle while the last one finishes (tools/xcd_diag.py: the XCDs' end times spread 8-29 %).
// The launch has list_grid() blocks (a multiple of 8 with 25 % slack); logical XCD j = b & 7 (the
// hardware deals blocks round-robin) takes the contiguous range [lo_j, lo_j+1) of the nb live
// blocks, lo_j = xcd_frac[j] * nb / 2^16 from DevState (k_xcd_split, from this step's search:
// a wave's work = its longest list + kWaveCost), and its blocks past the range exit.  Any range
// past the grid's share, or no split yet, falls back to the equal ranges of xcd_block: each live
// block is taken exactly once either way.  Returns the block's index among the live blocks, or -1.
// The search itself keeps the equal ranges: its cost follows the candidates it scans, not the
// lists it writes (balanced by list length it ran 8 % slower at D1M; by the previous step's wave
// durations all three kernels oscillated, profiles/r03/xcd_balance/).
constexpr int kWaveCost = 16;   // a wave's fixed cost, in list entries, for the work histogram

// rev: each XCD takes its range from the far end (pass A: it starts on the list tiles the search
// wrote last, which the Infinity Cache still holds)
__device__ __forceinline__ int list_block(const DevState* st, int n, bool rev = false)
{
    const int nb = list_blocks(n);
    const int b = blockIdx.x;
    if (st) {
        const int* fr = st->xcd_frac;
        const int cap = gridDim.x >> 3;
        const int j = b & 7;
        bool ok = fr[0] == 0 && fr[8] == 65536;
        int lo = 0, mine_lo = 0, mine_c = 0;
        for (int x = 0; x < 8; ++x) {
            const int hi = (int)(((long long)fr[x + 1] * nb) >> 16);
            const int c = hi - lo;
            ok = ok && c >= 0 && c <= cap;
            if (x == j) { mine_lo = lo; mine_c = c; }
            lo = hi;
        }
        if (ok) {
            const int q = b >> 3;
            return q < mine_c ? mine_lo + (rev ? mine_c - 1 - q : q) : -1;
        }
    }
    if (b >= nb) return -1;
    if (!rev) return xcd_block(b, nb);
    // xcd_block's range of XCD b & 7 from its end
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    const int lo = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    const int cnt = q + (xcd < r ? 1 : 0);
    return lo + cnt - 1 - (b >> 3);
}

// The search's contribution to the work histogram: its wave's longest list (all lanes converged;
// one atomic per wave, spread over the 4096 runs).
__device__ __forceinline__ void add_wave_work(DevState* st, int cnt, int i, int n)
{
    if (!st) return;
    int m = cnt;
    for (int o = 32; o; o >>= 1) m = max(m, __shfl_xor(m, o));
    const int tile = __builtin_amdgcn_readfirstlane(i >> 6);
    const int ntile = (n + 63) >> 6;
    if ((threadIdx.x & 63) == 0 && tile < ntile)
        atomicAdd(&st->seg_work[(int)(((long long)tile * kXcdSegs) / ntile)], m + kWaveCost);
}

__device__ __forceinline__ int nbr_entry(int j, int type) { return j | (type << kTypeShift); }
// The search's per-lane counter (scan_candidates_lds): lane x 4 in bits 0-7, the row of the next
// stored entry in bits 8-17 (the stored entries so far plus the gaps of the row jumps; up to 1023,
// so a lane that keeps all 512 entries the reference allows does not carry into the total) and
// every accepted neighbour from bit 18.  The next list slot's byte offset in the wave's ELL tile is
// soff & kSoffMask; a row past the tile's kTileRows (only an overflowing lane, > 512 entries, the
// step's MPH_ERR_NEIGHBOR_OVERFLOW) is dropped by the tile's buffer descriptor.
constexpr int kListKeep = 256 + (1 << 18), kListTotal = 1 << 18, kSoffMask = 0x3FFFF;
__device__ __forceinline__ int soff_total(int soff) { return (int)((unsigned)soff >> 18); }
__device__ __forceinline__ int soff_stored(int soff) { return (soff >> 8) & 0x3FF; }

// Pass B's gather record {x, y, z, PressureP} (Launch.rec) lives in two 16-byte planes: {x, y} of
// particle j at [j], {z, P} at [ps + j], ps = the array capacity (DevParams.n).  A 16-byte gather
// instruction of a wavefront then reads one plane: 64 lanes whose neighbours are consecutive
// particles touch 1 KB (8 lines of 128 B) instead of 2 KB of whole records (same box: D1M pass B
// 0.271 -> 0.251 ms, D16M 2.89 -> 2.66 ms, profiles/r05/planes/).  Pass A's 48-byte records
// {x, y, z, vx, vy, vz} (Soa.p6) stay whole: in three planes pass A lost (0.376 -> 0.446 ms).

// Velocity of sorted particle i for the list passes, from its gather record {x, y, z, vx, vy, vz}
// (k_rank_scatter then skips the SoA velocity stores).
__device__ __forceinline__ void own_velocity(const Soa& A, int i, double& vx, double& vy, double& vz)
{
    const double2 b = A.p6[3 * (size_t)i + 1], c = A.p6[3 * (size_t)i + 2];
    vx = b.y; vy = c.x; vz = c.y;
}

__device__ __forceinline__ const int* ell_row(const int* nbr, int i)
{
    return nbr + (size_t)(i >> 6) * kTileStride + (i & 63);
}

// entry k of a lane from the lane's ell_row pointer: row k of the wave's tile
__device__ __forceinline__ const int* ell_at(const int* row, int lane, int k)
{
    return row - lane + ell_slot(k, lane);
}

// The wave's ELL tile and the lane: entry k of the lane at row k, by a 32-bit byte offset from the
// tile's (SGPR) base -- one shift-or per entry instead of 64-bit address arithmetic.
struct NbrList {
    const int* tile;   // the wave's list tile (wave-uniform)
    int lane;
};

__device__ __forceinline__ NbrList nbr_list(const int* nbr, int i)
{
    NbrList L;
    L.tile = nbr + (size_t)__builtin_amdgcn_readfirstlane(i >> 6) * kTileStride;
    L.lane = i & 63;
    return L;
}

// entry k of the lane: neighbour index j and type t.  (A buffer descriptor here, to skip the loads
// past a lane's end, costs pass A 4 more SGPRs than it has: spills inside its loop.)
__device__ __forceinline__ void nbr_at(const NbrList& L, int k, int& j, int& t)
{
    using gcchar = const __attribute__((address_space(1))) char;
    using gcint = const __attribute__((address_space(1))) int;
    const int e = *(gcint*)((gcchar*)L.tile + ((unsigned)ell_slot(k, L.lane) << 2));
    j = e & kIndexMask;
    t = e >> kTypeShift;
}

// Aligned rows (mph_params.h kAlignRows).  A wave's jumps are recorded in two places: the wave's
// header word lhdr[tile] (byte k < kMaxJumps: the row the lanes moved on to at jump k; byte 7: the
// number of jumps J), and per lane lgap[i] (byte k: the lane's own row when it jumped), so the
// lane's gap k is the rows [lgap byte k, lhdr byte k).  Every row of [0, end) outside the gaps
// holds an entry (end = the lane's ncount), in the lane's list order.  A wave that never jumps
// (J = 0: on the lattice, and every wave of the per-lane search) has plain rows, entry k at row k.
// RowMask: the rows below kAlignRows that hold an entry, one bit each; rows from kAlignRows on
// hold one exactly when they are below end.
struct RowMask {
    unsigned long long lo, hi;
};

// bits [k, 64) of a 64-bit word, k clamped to [0, 64]
__device__ __forceinline__ unsigned long long bits_from(int k)
{
    return k <= 0 ? ~0ull : (k >= 64 ? 0ull : (~0ull << k));
}

__device__ __forceinline__ RowMask row_mask(unsigned long long hdr, const unsigned long long* lgap, int i, int end)
{
    RowMask m;
    m.lo = ~bits_from(end);
    m.hi = ~bits_from(end - 64);
    const int J = (int)(hdr >> 56);
    if (J) {   // wave-uniform
        const unsigned long long g = lgap[i];
        for (int k = 0; k < J; ++k) {
            const int a = (int)((g >> (8 * k)) & 0xff), b = (int)((hdr >> (8 * k)) & 0xff);
            m.lo &= ~(bits_from(a) & ~bits_from(b));
            m.hi &= ~(bits_from(a - 64) & ~bits_from(b - 64));
        }
    }
    return m;
}

// whether row r holds one of the lane's entries
__device__ __forceinline__ bool row_ok(const RowMask& m, int r, int end)
{
    if (r < 64) return (m.lo >> r) & 1;
    if (r < kAlignRows) return (m.hi >> (r - 64)) & 1;
    return r < end;
}

// rows [k0 + a, k0 + b) as bits 0..31, a, b clamped to [0, 32]
__device__ __forceinline__ unsigned bit_range(int a, int b)
{
    auto low = [](int n) { return n <= 0 ? 0u : (n >= 32 ? ~0u : (1u << n) - 1u); };
    return low(b) & ~low(a);
}

// the rows from kAlignRows on: bit u set when row k0 + u holds an entry there (k0 + u < end)
__device__ __forceinline__ unsigned tail_bits(int k0, int end)
{
    return bit_range(kAlignRows - k0, end - k0);
}

// bit u: row k0 + u holds one of the lane's entries (k0 wave-uniform in the list loops; bits
// 0..31), without branches
__device__ __forceinline__ unsigned row_bits(const RowMask& m, int k0, int end)
{
    const int k = k0 < kAlignRows ? k0 : kAlignRows - 1;
    const unsigned long long lo = k < 64 ? m.lo : m.hi, hi = k < 64 ? m.hi : 0ull;
    const int sh = k & 63;
    const unsigned b = (unsigned)((lo >> sh) | (sh ? hi << (64 - sh) : 0ull));
    return (b & bit_range(0, kAlignRows - k0)) | tail_bits(k0, end);
}

// The 128 mask bits of the lanes of a wave in LDS, 6 dwords per lane (the last two zero; a 24-byte
// stride keeps the 32 lanes of a read group on distinct banks): pass A, whose registers are full
constexpr int kMaskWords = 6;
__device__ __forceinline__ void mask_to_lds(unsigned* lm, const RowMask& m)
{
    lm[0] = (unsigned)m.lo;
    lm[1] = (unsigned)(m.lo >> 32);
    lm[2] = (unsigned)m.hi;
    lm[3] = (unsigned)(m.hi >> 32);
    lm[4] = 0u;
    lm[5] = 0u;
}
__device__ __forceinline__ unsigned row_bits_lds(const unsigned* lm, int k0, int end)
{
    const int d = k0 < kAlignRows ? k0 >> 5 : 3;
    const unsigned long long v = (unsigned long long)lm[d] | ((unsigned long long)lm[d + 1] << 32);
    return ((unsigned)(v >> (k0 & 31)) & bit_range(0, kAlignRows - k0)) | tail_bits(k0, end);
}


// the wave's header word (scalar load)
__device__ __forceinline__ unsigned long long wave_hdr(const unsigned long long* lhdr, int i)
{
    return lhdr[__builtin_amdgcn_readfirstlane(i >> 6)];
}

// The search's row jumps: a jump at a stencil group end only when the wave's rows have drifted at
// least this far apart (highest - lowest row of the live lanes); 1 = at every group end where the
// rows differ, a value > kAlignRows = never (plain rows)
#ifndef MPH_PASS_A_REV
#define MPH_PASS_A_REV 1
#endif
#ifndef MPH_ALIGN_DRIFT
#define MPH_ALIGN_DRIFT 1
#endif
constexpr int kAlignDrift = MPH_ALIGN_DRIFT;

// ------------------------------------------------------------------------- sort phase -------

// calculateWall (main.cpp:3031-3060) + calculatePeriodicBoundary (3322-3333) + cell histogram.
// mode 0: initialisation (no motion), 1: time step, 2: time step whose motion was already applied
// (slab mode, k_dist_prep).
// calculateWall (3031-3060) then calculatePeriodicBoundary (3322-3333) for particle p of B.
__device__ __forceinline__ void move_and_wrap(const DevParams& P, const DevState* st, Soa& B, int p,
                                              double& x, double& y, double& z)
{
#pragma clang fp contract(off)
    const int t = B.type[p];
    if (P.module == MPH_MODULE_TUREK_HRON && dev_is_fluid(t)) {
        // Turek_Hron: setInitialVelocityProfile (main.cpp:419-441) runs every step before
        // calculateWall (592-594): parabolic inlet for x <= 0.01 and, while Time < 0.7, the same
        // profile (without the 1.5 factor) for x > 1.5; YMIN/YMAX/UMAX from main.cpp:374-377
        const double ymin = 0.0, ymax = 0.41, umax = 1.0, h = ymax - ymin;
        if (x <= 0.01) {
            const double uy = y - ymin;
            B.vx[p] = (1.5 * 4.0 * umax / (h * h)) * uy * (h - uy);
            B.vy[p] = 0.0;
            B.vz[p] = 0.0;
        }
        if (x > 1.5 && st->time < 0.7) {
            const double uy = y - ymin;
            B.vx[p] = (4.0 * umax / (h * h)) * uy * (h - uy);
            B.vy[p] = 0.0;
            B.vz[p] = 0.0;
        }
    }
    if (dev_is_wall(t) && P.wall_motion == MPH_WALL_ROLLING) {
        // the Rolling branch of calculateWall (main.cpp:2974-3022): rotate about z through
        // WallCenter by the step's angle increment; the velocity is omega(t) x r_rot
        const double max_angle = 2.0 * M_PI / 180.0, period = 1.646;   // main.cpp:2959-2960
        const double omega_t = 2.0 * M_PI / period;
        const double theta = max_angle * sin(omega_t * st->time);
        const double dtheta_dt = max_angle * omega_t * cos(omega_t * st->time);
        const double theta_prev = max_angle * sin(omega_t * (st->time - P.dt));
        const double delta_theta = theta - theta_prev;
        const double cosD = cos(delta_theta), sinD = sin(delta_theta);
        const double* C = st->wall_c[t];
        const double r0 = x - C[0], r1 = y - C[1], r2 = z - C[2];
        const double a0 = cosD * r0 + -sinD * r1;
        const double a1 = sinD * r0 + cosD * r1;
        const double a2 = r2;
        const double w0 = 0.0, w1 = 0.0, w2 = dtheta_dt;
        B.vx[p] = w1 * a2 - w2 * a1;
        B.vy[p] = w2 * a0 - w0 * a2;
        B.vz[p] = w0 * a1 - w1 * a0;
        x = a0 + C[0];
        y = a1 + C[1];
        z = a2 + C[2];
    } else if (dev_is_wall(t) && st->time < 0.2) {
        const double* C = st->wall_c[t];
        const double* V = st->wall_vel[t];
        const double* w = st->wall_omega[t];
        const double (*R)[3] = st->wall_rot[t];
        const double r0 = x - C[0], r1 = y - C[1], r2 = z - C[2];
        const double a0 = R[0][0] * r0 + R[0][1] * r1 + R[0][2] * r2;
        const double a1 = R[1][0] * r0 + R[1][1] * r1 + R[1][2] * r2;
        const double a2 = R[2][0] * r0 + R[2][1] * r1 + R[2][2] * r2;
        B.vx[p] = w[1] * a2 - w[2] * a1 + V[0];
        B.vy[p] = w[2] * a0 - w[0] * a2 + V[1];
        B.vz[p] = w[0] * a1 - w[1] * a0 + V[2];
        x = a0 + C[0] + V[0] * P.dt;
        y = a1 + C[1] + V[1] * P.dt;
        z = a2 + C[2] + V[2] * P.dt;
    }
    x = mod_exact(x - P.dmin[0], P.dw[0]) + P.dmin[0];
    y = mod_exact(y - P.dmin[1], P.dw[1]) + P.dmin[1];
    z = mod_exact(z - P.dmin[2], P.dw[2]) + P.dmin[2];
    B.x[p] = x;
    B.y[p] = y;
    B.z[p] = z;
}

// entry p of a sort input C: its set (C or the VSrc's V) and index there; mig: a kept migrant
// (its id is read negated)
__device__ __forceinline__ int vsrc_entry(const VSrc& vs, const Soa& C, int p, Soa& S, bool& mig)
{
    S = C;
    mig = false;
    if (vs.idx && p < *vs.n) {
        const int q = vs.idx[p];
        mig = q < 0;
        S = vs.V;
        return mig ? -1 - q : q;
    }
    return p;
}

constexpr int kScanThreads = 256;
#ifndef MPH_SCAN_ITEMS
#define MPH_SCAN_ITEMS 16
#endif
constexpr int kScanItems = MPH_SCAN_ITEMS;   // cells per thread (a multiple of 4)
constexpr int kScanBlock = kScanThreads * kScanItems;   // 4096 cells per block
// ints of the scan's block totals (mph_ctx.hip allocates them)
__host__ __device__ inline int bsum_stride(int ncell) { return ncell / kScanBlock + 2; }
static_assert(kScanBlock == 4096, "mph_ctx.hip sizes the bsum buffer for 4096-cell blocks");

// The XCD split of the list passes (see list_block) from the search's work histogram: an inclusive
// scan of the runs' work (kXcdSegs / blockDim.x consecutive runs per thread), the 7 inner cut
// points at equal shares of the total (interpolated inside their run), then the histogram cleared.
// Block 0 of the next step's k_rank_scatter calls it (see there).
template <int T>
__device__ __forceinline__ void xcd_split_block(DevState* st)
{
    constexpr int R = kXcdSegs / T;
    static_assert(kXcdSegs % T == 0, "whole runs per thread");
    __shared__ long long s[T];
    const int t = threadIdx.x;
    long long sum = 0;
    for (int r = 0; r < R; ++r) sum += max(st->seg_work[t * R + r], 0);
    s[t] = sum;
    __syncthreads();
    for (int o = 1; o < T; o <<= 1) {
        const long long v = t >= o ? s[t - o] : 0;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    const long long tot = s[T - 1];
    int* fr = st->xcd_frac;
    if (tot < 8) {
        if (t < 9) fr[t] = 8192 * t;
    } else {
        for (int x = 1; x < 8; ++x) {
            const long long tgt = tot * x / 8;
            long long prev = t ? s[t - 1] : 0;
            if (!(prev < tgt && s[t] >= tgt)) continue;
            for (int r = 0; r < R; ++r) {
                const int w = max(st->seg_work[t * R + r], 0);
                if (w > 0 && prev < tgt && prev + w >= tgt) {
                    const double f = (t * R + r + (double)(tgt - prev) / (double)w) / kXcdSegs;
                    fr[x] = min(65536, max(0, (int)(f * 65536.0 + 0.5)));
                }
                prev += w;
            }
        }
        if (t == 0) {
            fr[0] = 0;
            fr[8] = 65536;
        }
    }
    __syncthreads();   // every thread has read its runs
    for (int r = 0; r < R; ++r) st->seg_work[t * R + r] = 0;
}

__global__ __launch_bounds__(256) void k_prep(DevParams P, const DevState* __restrict__ st, Soa C,
                                              int* __restrict__ key, int* __restrict__ slot,
                                              int* __restrict__ cnt, int mode, VSrc vs)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = dev_n(P);
    Soa B = C;
    bool mig = false;
    const int b = p < n ? vsrc_entry(vs, C, p, B, mig) : p;
    {
        // The particles arrive in the previous cell order, so consecutive lanes often share a
        // cell: one histogram atomic per run of equal keys (slot = run base + rank in the run).
        // Every lane of the wave takes part in the shuffles; lanes past n form runs of their own.
        const bool live = p < n;
        int k = -1 - (int)(threadIdx.x & 63);
        int occ = 0;
        if (live) {
            double x = B.x[b], y = B.y[b], z = B.z[b];
            if (mode == 1) move_and_wrap(P, st, B, b, x, y, z);
            if (!isfinite(x + y + z)) atomicOr(const_cast<int*>(&st->overflow), 4);   // MPH_ERR_NONFINITE
            k = cell_id(P, x, y, z);
            key[p] = k;
            occ = seam_bits(P, x, y, z);
        }
        const int lane = threadIdx.x & 63;
        const int kprev = __shfl_up(k, 1, 64);
        const bool head = lane == 0 || kprev != k;
        const unsigned long long heads = __ballot(head);
        const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
        const int hl = 63 - __clzll(heads & upto);
        const unsigned long long above = heads & ~upto;
        const int next = above ? __ffsll((long long)above) - 1 : 64;
        int base = 0;
        if (live && head) base = atomicAdd(&cnt[k], next - lane);
        base = __shfl(base, hl, 64);
        if (live) slot[p] = base + (lane - hl);
        // the block's face bits: OR-ed in LDS, then one device atomic per block, only for bits the
        // step's word does not hold yet (few blocks: the particles near a periodic face)
        __shared__ int s_occ;
        if (threadIdx.x == 0) s_occ = 0;
        __syncthreads();
        if (__ballot(occ != 0)) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) occ |= __shfl_xor(occ, o, 64);
            if (lane == 0) atomicOr(&s_occ, occ);
        }
        __syncthreads();
        if (threadIdx.x == 0 && s_occ) {
            int* w = const_cast<int*>(&st->seam_occ[st->seam_step & 1]);
            const int cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (s_occ & ~cur) atomicOr(w, s_occ);
        }
    }
}

// Exclusive scan of the cell histogram (constants above k_prep): block totals (k_scan_reduce), the
// top-level scan (inside k_scan_down up to kScanFusedTop blocks, else a
// k_scan_top launch) and the down-sweep.

__device__ __forceinline__ int block_exclusive_scan(int v, int* lds, int& total)
{
    // wave-level inclusive scan (64 lanes) + cross-wave via LDS
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    int wsum = 0;
    const int nw = blockDim.x >> 6;
    total = 0;
    for (int w = 0; w < nw; ++w) {
        const int s = lds[w];
        if (w < wid) wsum += s;
        total += s;
    }
    __syncthreads();
    return wsum + x - v;
}

// 16 consecutive counts of one thread: four 16-byte loads when the run is inside the array
// (cell arrays are 16-int aligned per thread), element loads at the tail.
__device__ __forceinline__ void load16(const int* __restrict__ a, int base, int n, int (&v)[kScanItems])
{
    if (base + kScanItems <= n) {
        const int4* q = reinterpret_cast<const int4*>(a + base);
#pragma unroll
        for (int k = 0; k < kScanItems / 4; ++k) {
            const int4 t = q[k];
            v[4 * k] = t.x; v[4 * k + 1] = t.y; v[4 * k + 2] = t.z; v[4 * k + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k) v[k] = base + k < n ? a[base + k] : 0;
    }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const int* __restrict__ cnt, int ncell,
                                                              int* __restrict__ bsum)
{
    __shared__ int lds[kScanThreads / 64];
    const int base = blockIdx.x * kScanBlock + threadIdx.x * kScanItems;
    int v[kScanItems];
    load16(cnt, base, ncell, v);
    int s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) s += v[k];
    int total;
    block_exclusive_scan(s, lds, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_scan_top(int* __restrict__ bsum, int nb)
{
    // each thread a run of R consecutive totals: its sum, one block scan of the sums, then the
    // run's exclusive prefixes (one round trip to memory instead of nb / blockDim.x of them)
    __shared__ int lds[16];
    const int t = threadIdx.x;
    const int R = (nb + (int)blockDim.x - 1) / (int)blockDim.x;
    const int b0 = min(nb, t * R), b1 = min(nb, b0 + R);
    int sum = 0;
#pragma unroll 8
    for (int b = b0; b < b1; ++b) sum += bsum[b];
    int total;
    int run = block_exclusive_scan(sum, lds, total);
#pragma unroll 8
    for (int b = b0; b < b1; ++b) {
        const int v = bsum[b];
        bsum[b] = run;
        run += v;
    }
}

// top: bsum holds the raw block totals and every block sums its predecessors' itself (no
// k_scan_top launch; used while the block count is small, kScanFusedTop)
#ifndef MPH_SCAN_FUSED_TOP
#define MPH_SCAN_FUSED_TOP 8192   // (the D16M / 8 slab ranks: no k_scan_top launch)
#endif
constexpr int kScanFusedTop = MPH_SCAN_FUSED_TOP;
__global__ __launch_bounds__(kScanThreads) void k_scan_down(int* __restrict__ cnt, int ncell,
                                                            const int* __restrict__ bsum,
                                                            int* __restrict__ start, int n,
                                                            const int* __restrict__ n_dev, int top)
{
    __shared__ int lds[kScanThreads / 64];
    const int base = blockIdx.x * kScanBlock + threadIdx.x * kScanItems;
    int v[kScanItems];
    load16(cnt, base, ncell, v);
    int pre = 0;
    if (top) {
        int t = 0;
        for (int b = threadIdx.x; b < (int)blockIdx.x; b += kScanThreads) t += bsum[b];
        block_exclusive_scan(t, lds, pre);
    } else {
        pre = bsum[blockIdx.x];
    }
    int s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) s += v[k];
    int total;
    int run = block_exclusive_scan(s, lds, total) + pre;
    int o[kScanItems];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        o[k] = run;
        run += v[k];
    }
    if (base + kScanItems <= ncell) {
        int4* st = reinterpret_cast<int4*>(start + base);
        int4* ct = reinterpret_cast<int4*>(cnt + base);
#pragma unroll
        for (int k = 0; k < kScanItems / 4; ++k) {
            st[k] = make_int4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
            // histogram ready for the next step; all-zero runs of 16 cells (most of the D1M tank is
            // empty, ~7 cells per particle) are left alone, so their lines are not written
            if (s != 0) ct[k] = make_int4(0, 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k)
            if (base + k < ncell) {
                start[base + k] = o[k];
                if (v[k] != 0) cnt[base + k] = 0;
            }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) start[ncell] = n_dev ? *n_dev : n;
}

// Unordered placement; block 0 also advances Time and WallCenter (main.cpp:685, 3066-3070)
// after k_prep consumed them.
__global__ __launch_bounds__(256) void k_place(DevParams P, DevState* __restrict__ st,
                                               const int* __restrict__ key, const int* __restrict__ slot,
                                               const int* __restrict__ start, int* __restrict__ tmp,
                                               int mode)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // this step's face bits are complete (k_prep): the searches read them; the next step's
        // k_prep gathers into the other word
        st->seam_occ[(st->seam_step + 1) & 1] = 0;
        st->seam_step += 1;
        if (mode) {
#pragma clang fp contract(off)
            for (int t = 4; t < 6; ++t)
                for (int d = 0; d < 3; ++d) st->wall_c[t][d] += st->wall_vel[t][d] * P.dt;
            st->time += P.dt;
        }
    }
    const int n = dev_n(P);
    if (p >= n) return;
    // a histogram inconsistent with the keys (it cannot happen while the block totals and the
    // counts agree) becomes an error flag, never a store out of range
    const int d = start[key[p]] + slot[p];
    if ((unsigned)d >= (unsigned)n) {
        atomicOr(&st->overflow, 64);
        return;
    }
    tmp[d] = p;
}

// Deterministic stable order inside a cell: rank = number of cell-mates with a smaller previous
// sorted index.  Reorders the persistent particle state into the new cell order.
__global__ __launch_bounds__(256) void k_rank_scatter(DevParams P, const int* __restrict__ key,
                                                      const int* __restrict__ start,
                                                      const int* __restrict__ tmp, Soa C, Soa A,
                                                      int* __restrict__ rank_of, int* __restrict__ dst_of,
                                                      int mode, VSrc vs, DevState* __restrict__ st, int split)
{
    // The passes' XCD split (list_block) runs here, in block 0 of the longest sort kernel, from
    // the previous step's search: a wave's work changes little from one step to the next and the
    // map only decides which block runs which wave, so no launch of its own sits between the
    // search and pass A (its own launch after the search cost 0.45 % at rest, 0.24 % developed,
    // profiles/r05/split_in_sort/)
    if (split && blockIdx.x == 0) xcd_split_block<256>(st);
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= dev_n(P)) return;
    const int k = key[p];
    const int s = start[k], e = start[k + 1];
    int r = 0;
    for (int q = s; q < e; ++q) r += tmp[q] < p;
    const int dst = s + r;
    Soa B;
    bool mig;
    const int b = vsrc_entry(vs, C, p, B, mig);
    A.x[dst] = B.x[b];
    A.y[dst] = B.y[b];
    A.z[dst] = B.z[b];
    // the sorted velocities are read only through the 48-byte records (own_velocity), except at a
    // slab context's initialisation sort (mode 0: dist_init copies the sorted set into B)
    if (dst_of && mode == 0) {
        A.vx[dst] = B.vx[b];
        A.vy[dst] = B.vy[b];
        A.vz[dst] = B.vz[b];
    }
    A.type[dst] = B.type[b];
    const int id = mig ? -1 - B.id[b] : B.id[b];
    A.id[dst] = id;
    A.p6[3 * (size_t)dst] = make_double2(B.x[b], B.y[b]);
    A.p6[3 * (size_t)dst + 1] = make_double2(B.z[b], B.vx[b]);
    A.p6[3 * (size_t)dst + 2] = make_double2(B.vy[b], B.vz[b]);
    A.f4[dst] = make_float4((float)(B.x[b] - P.cref[0]), (float)(B.y[b] - P.cref[1]),
                            (float)(B.z[b] - P.cref[2]), __int_as_float(B.type[b]));
    if (dst_of) dst_of[p] = dst;   // slab mode: ids are global (ghosts negative)
    else if (rank_of) rank_of[id] = dst;
}

// ----------------------------------------------------------------------------- pass A sums --

struct PassA {
    double da = 0.0, g0 = 0.0, g1 = 0.0, g2 = 0.0, vs = 0.0, dv = 0.0;
    // force sums that need no pass-A value of j: S = sum_j [r<RP] dwp(r)/r V q_ij (the P_i half
    // of calculatePressureP's (P_i+P_j) term, 2394-2424) and the viscous force (2478-2522)
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, v0 = 0.0, v1 = 0.0, v2 = 0.0;
};

// One neighbour's contribution to DensityA (2141-2171), GravityCenter (2174-2210), DensityP
// (2314-2341), DivergenceP (2343-2379), and (FORCE) the P_i half of the pressure force and the
// viscous force; (dvx, dvy, dvz) = v_j - v_i.  No implicit contraction: every accumulation is an
// explicit fma, so this branching form and the selecting form of the round-3 fused kernel
// give the same bits (a deselected fma(a, 0, acc) leaves acc unchanged).
template <bool FORCE, bool EQR = false>
__device__ __forceinline__ void pass_a_term(const DevParams& P, const double* s_ratio, const double* s_mu, int ti,
                                            int tj, bool solid, double q0, double q1, double q2, double r2,
                                            double dvx, double dvy, double dvz, PassA& o)
{
#pragma clang fp contract(off)
    double r, ir;
    rsqrt_pair(r2, r, ir);
    const double dot = fma(dvz, q2, fma(dvy, q1, dvx * q0));
    if (EQR) {
        // RadiusA = RadiusP = RadiusV (pass_a_equal_radii): one cutoff test and one 1 - r/h for
        // all four kernels; same expressions otherwise
        if (r2 <= P.rp2) {
            const double t = r * P.inv_rp;
            const double omt = 1.0 - t;
            const double omt2 = omt * omt;
            const double u = (P.cdp * omt) * ir;
            o.vs = fma(P.cp, omt2, o.vs);
            o.dv = fma(-dot, u, o.dv);
            const bool strict = r2 < P.rp2;
            if (FORCE && strict && !(solid && dev_is_struct(tj))) {
                const double c = u * P.vol;
                o.s0 = fma(c, q0, o.s0);
                o.s1 = fma(c, q1, o.s1);
                o.s2 = fma(c, q2, o.s2);
            }
            if (!solid) {
                const double ratio = s_ratio[ti * kTypes + tj];
                o.da = fma(ratio, (P.ca * t) * omt2, o.da);
                const double w = (ratio * (P.cg * omt2)) * P.rg_r2g;
                o.g0 = fma(q0, w, o.g0);
                o.g1 = fma(q1, w, o.g1);
                o.g2 = fma(q2, w, o.g2);
                if (FORCE && strict) {
                    const double c = ((s_mu[ti * kTypes + tj] * omt) * dot) * ((ir * ir) * ir);
                    o.v0 = fma(c, q0, o.v0);
                    o.v1 = fma(c, q1, o.v1);
                    o.v2 = fma(c, q2, o.v2);
                }
            }
        }
        return;
    }
    if (r2 <= P.rp2) {
        const double omt = 1.0 - r * P.inv_rp;
        const double u = (P.cdp * omt) * ir;   // dw_p(r) / r
        o.vs = fma(P.cp * omt, omt, o.vs);
        o.dv = fma(-dot, u, o.dv);
        // strict test of the force loops (2402), and structure i sees only non-structure j
        // (InterfaceForce 2439-2472)
        if (FORCE && r2 < P.rp2 && !(solid && dev_is_struct(tj))) {
            const double c = u * P.vol;
            o.s0 = fma(c, q0, o.s0);
            o.s1 = fma(c, q1, o.s1);
            o.s2 = fma(c, q2, o.s2);
        }
    }
    if (!solid) {
        const double ratio = s_ratio[ti * kTypes + tj];
        if (r2 <= P.ra2) {
            const double t = r * P.inv_ra;
            const double omt = 1.0 - t;
            o.da = fma(ratio, ((P.ca * t) * omt) * omt, o.da);
        }
        if (r2 <= P.rg2) {
            const double omt = 1.0 - r * P.inv_rg;
            const double w = (ratio * ((P.cg * omt) * omt)) * P.rg_r2g;
            o.g0 = fma(q0, w, o.g0);
            o.g1 = fma(q1, w, o.g1);
            o.g2 = fma(q2, w, o.g2);
        }
        if (FORCE && r2 < P.rv2) {
            // s_mu holds -cvis cdv vol mu_ij (k_pass_a): dw_v(r) = -cdv (1 - r / rv)
            const double c = ((s_mu[ti * kTypes + tj] * (1.0 - r * P.inv_rv)) * dot) * ((ir * ir) * ir);
            o.v0 = fma(c, q0, o.v0);
            o.v1 = fma(c, q1, o.v1);
            o.v2 = fma(c, q2, o.v2);
        }
    }
}

// Epilogue: PhysicalCoefficients (2099-2137) and the pressure values of calculatePressureP
// (2384-2392) and calculatePressureA (2218-2223); with fpart, the neighbour-independent part of
// the force P_i S_i + viscous force, and the pass-B gather record {x, y, z, P}.
struct PassAOut {
    double *pres, *gx, *gy, *gz, *pa, *dens_a, *vstrain, *divp;
    double4 *fpart, *rec;
};

// pass B's gather record {x, y, z, PressureP} of sorted particle i (planes {x, y} and {z, P}, see
// above; ps = DevParams.n), and its PressureP alone (the halo)
__device__ __forceinline__ void rec_store(double4* rec, int ps, int i, double x, double y, double z, double p)
{
    double2* r = reinterpret_cast<double2*>(rec);
    r[i] = make_double2(x, y);
    r[(size_t)ps + i] = make_double2(z, p);
}
__device__ __forceinline__ void rec_store_p(double4* rec, int ps, int i, double p)
{
    reinterpret_cast<double2*>(rec)[(size_t)ps + i].y = p;
}
__device__ __forceinline__ void rec_load(const double4* rec, int ps, int j, double& x, double& y, double& z, double& p)
{
    const double2* r = reinterpret_cast<const double2*>(rec);
    const double2 a = r[j], b = r[(size_t)ps + j];
    x = a.x; y = a.y; z = b.x; p = b.y;
}

__device__ __forceinline__ void pass_a_finish(const DevParams& P, const DevTables* T, int ti, int i,
                                              const PassA& o, const PassAOut& out, double xi = 0.0,
                                              double yi = 0.0, double zi = 0.0)
{
    const double vstr = o.vs - P.n0p;
    const double kappa = vstr < 0.0 ? 0.0 : T->bulk[ti];
    double p = -T->bulk_visc[ti] * o.dv;
    if (vstr > 0.0) p += kappa * vstr;
    double pa = T->cofa[ti] * (o.da - P.n0a) / P.dx;
    if (P.n0a <= o.da) pa = 0.0;
    out.pres[i] = p;
    // null on the non-last steps of a replayed batch when nothing downstream reads them
    // (enqueue_step): GravityCenter/PressureA without surface tension, the three diagnostics
    if (out.gx) {
        out.gx[i] = o.g0;
        out.gy[i] = o.g1;
        out.gz[i] = o.g2;
        out.pa[i] = pa;
    }
    if (out.dens_a) {
        out.dens_a[i] = o.da;
        out.vstrain[i] = vstr;
        out.divp[i] = o.dv;
    }
    if (out.fpart) {
        out.fpart[i] = make_double4(p * o.s0 + o.v0, p * o.s1 + o.v1, p * o.s2 + o.v2, 0.0);
        rec_store(out.rec, P.n, i, xi, yi, zi, p);
    }
}

// ---------------------------------------------------------------------- neighbour search ----

// calculateNeighbor (main.cpp:1743-1810).  The reference scans (2*3+1)^d cells of width dx; here
// cells are >= rc/kReach (rc/3) wide across the two column axes and >= rc/kContigReach (rc/2)
// along the contiguous one, so a +-kReach stencil covers the acceptance sphere: (2 kReach + 1)^2
// = 49 columns (3-D) or 7 (2-D), each one contiguous index range of +-kContigReach cells of the
// last axis.  Acceptance is the reference's own test  q0^2+q1^2+q2^2 <= (MaxRadius+MARGIN)^2
// with the Mod-based minimum image.
// Offset of x from the grid origin, wrapped once into [0, w) (as cell_axis).
__device__ __forceinline__ double grid_offset(double x, double org, double w)
{
    const double u = x - org;
    return u < 0.0 ? u + w : (u >= w ? u - w : u);
}

// Gap between grid offset u (inside cell c) and cell c + d along one axis (0 for d == 0).
__device__ __forceinline__ double cell_gap(double u, int c, int d, double cw)
{
    const double g = d > 0 ? (c + d) * cw - u : (d < 0 ? u - (c + d + 1) * cw : 0.0);
    return g > 0.0 ? g : 0.0;
}

// calculateNeighbor's acceptance (main.cpp:1760-1765) for an interior pair, bit-exact but cheap:
// r2 from the raw difference d = x_j - x_i (FMA) differs from the reference's
// q = (d + W/2) - W/2, r2 = q0^2+q1^2+q2^2 by < 1e-13 relative, so outside a +-1e-10 band
// around rc^2 the answer is decided; inside it (rare) the reference expression is evaluated.
__device__ __forceinline__ bool accept_interior(const DevParams& P, double dx, double dy, double dz,
                                                double lo2, double hi2)
{
    const double r2a = fma(dx, dx, fma(dy, dy, dz * dz));
    bool a = r2a <= lo2;
    if (!a && r2a <= hi2) {   // two compares: the band is "<= hi2 and not <= lo2"
        const double q0 = image_exact<true>(dx, P.dw[0], P.hw[0], P.w075[0]);
        const double q1 = image_exact<true>(dy, P.dw[1], P.hw[1], P.w075[1]);
        const double q2 = image_exact<true>(dz, P.dw[2], P.hw[2], P.w075[2]);
        a = r2_exact(q0, q1, q2) <= P.rc2;
    }
    return a;
}

// the reference's own acceptance expression (as accept_interior inside its band)
__device__ __forceinline__ bool accept_band(const DevParams& P, double dx, double dy, double dz)
{
    const double q0 = image_exact<true>(dx, P.dw[0], P.hw[0], P.w075[0]);
    const double q1 = image_exact<true>(dy, P.dw[1], P.hw[1], P.w075[1]);
    const double q2 = image_exact<true>(dz, P.dw[2], P.hw[2], P.w075[2]);
    return r2_exact(q0, q1, q2) <= P.rc2;
}

template <int DIM, bool FAST, int PERM, int SB = MPH_SB>
__device__ __forceinline__ int scan_candidates(const DevParams& P, const Soa& A, const int* start,
                                               int i, double xi, double yi, double zi, int cx,
                                               int cy, int cz, int* out)
{
    using X = CellAxes<DIM, PERM>;
    int cnt = 0;
    constexpr int NCOL = DIM == 3 ? kGroups * kGroups : kGroups;
    const int cc[3] = {cx, cy, cz};
    const int gca = P.gc[X::A2];   // contiguous axis
    const int cca = cc[X::A2];
    // Column trimming: skip the cells of a column (and whole columns) that lie entirely beyond
    // the cutoff.  Conservative (cutoff enlarged by 1e-6 relative, far above the roundoff of the
    // cell geometry), so the accepted set and its order are unchanged.
    const double rcm2 = P.rc2_trim;
    const double cw0 = P.cwid[X::A0], cw1 = P.cwid[X::A1];
    const double uu[3] = {grid_offset(xi, P.corg[0], P.dw[0]), grid_offset(yi, P.corg[1], P.dw[1]),
                          DIM == 3 ? grid_offset(zi, P.corg[2], P.dw[2]) : 0.0};
    const double ua = uu[X::A2];                      // offset along the contiguous axis
    const double lo2 = P.rc2_lo, hi2 = P.rc2_hi;
    const double ginva = P.ginv[X::A2];
    for (int col = 0; col < NCOL; ++col) {
        int base;
        double d2;
        if (DIM == 3) {
            const int dxc = col / kGroups - kReach, dyc = col % kGroups - kReach;
            const int c0 = cc[X::A0], c1 = cc[X::A1];
            const double gx = cell_gap(uu[X::A0], c0, dxc, cw0), gy = cell_gap(uu[X::A1], c1, dyc, cw1);
            d2 = gx * gx + gy * gy;
            if (d2 > rcm2) continue;
            const int jx = FAST ? c0 + dxc : wrap_cell(c0 + dxc, P.gc[X::A0]);
            const int jy = FAST ? c1 + dyc : wrap_cell(c1 + dyc, P.gc[X::A1]);
            base = (jx * P.gc[X::A1] + jy) * P.gc[X::A2];
        } else {
            const int dxc = col - kReach;
            const double gx = cell_gap(uu[0], cx, dxc, cw0);
            d2 = gx * gx;
            if (d2 > rcm2) continue;
            base = (FAST ? cx + dxc : wrap_cell(cx + dxc, P.gc[0])) * P.gc[1];
        }
        const double ra = sqrt(rcm2 - d2);
        const int lo = (int)fmax(floor((ua - ra) * ginva), (double)(cca - P.sa));
        const int hi = (int)fmin(floor((ua + ra) * ginva), (double)(cca + P.sa));
        int seg_a[2], seg_b[2], nseg;
        if (FAST) { seg_a[0] = lo; seg_b[0] = hi; seg_a[1] = 0; seg_b[1] = -1; nseg = 1; }
        else if (lo < 0) { seg_a[0] = lo + gca; seg_b[0] = gca - 1; seg_a[1] = 0; seg_b[1] = hi; nseg = 2; }
        else if (hi >= gca) { seg_a[0] = lo; seg_b[0] = gca - 1; seg_a[1] = 0; seg_b[1] = hi - gca; nseg = 2; }
        else { seg_a[0] = lo; seg_b[0] = hi; seg_a[1] = 0; seg_b[1] = -1; nseg = 1; }
        for (int sg = 0; sg < nseg; ++sg) {
            const int jb = start[base + seg_a[sg]];
            const int je = start[base + seg_b[sg] + 1];
            // batches of SB candidates: all loads issued before the first test (memory-level
            // parallelism; the loop is bound by the gathers, not by the FP64 arithmetic)
            for (int j0 = jb; j0 < je; j0 += SB) {
                double xs[SB], ys[SB], zs[SB];
                {
#pragma unroll
                    for (int u = 0; u < SB; ++u) {
                        const int j = j0 + u < je ? j0 + u : je - 1;
                        xs[u] = A.x[j];
                        ys[u] = A.y[j];
                        zs[u] = A.z[j];
                    }
                }
#pragma unroll
                for (int u = 0; u < SB; ++u) {
                    const int j = j0 + u;
                    bool a;
                    if (FAST) {
                        a = accept_interior(P, xs[u] - xi, ys[u] - yi, zs[u] - zi, lo2, hi2);
                    } else {
                        const double q0 = image_exact<false>(xs[u] - xi, P.dw[0], P.hw[0], P.w075[0]);
                        const double q1 = image_exact<false>(ys[u] - yi, P.dw[1], P.hw[1], P.w075[1]);
                        const double q2 = image_exact<DIM == 2>(zs[u] - zi, P.dw[2], P.hw[2], P.w075[2]);
                        a = r2_exact(q0, q1, q2) <= P.rc2;
                    }
                    if (a && j < je && j != i) {
                        if (cnt < kMaxNeighbor) out[ell_slot(cnt, 0)] = nbr_entry(j, A.type[j]);
                        ++cnt;
                    }
                }
            }
        }
    }
    return cnt;
}

// Wave-wide min / max (result in every lane).  DPP form: shifts within 16-lane rows, then
// row_bcast:15 / :31 carry the partial results across rows (gfx9 family), lane 63 holds the
// total; 7 dependent VALU steps instead of 6 dependent LDS permutes.
template <bool MAX>
__device__ __forceinline__ int wave_reduce_dpp(int v)
{
    const int id = MAX ? INT_MIN : INT_MAX;
    auto op = [](int a, int b) { return MAX ? max(a, b) : min(a, b); };
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x113, 0xf, 0xf, false));   // row_shr:3
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x114, 0xf, 0xe, false));   // row_shr:4
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x118, 0xf, 0xc, false));   // row_shr:8
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int wave_min(int v) { return wave_reduce_dpp<false>(v); }
__device__ __forceinline__ int wave_max(int v) { return wave_reduce_dpp<true>(v); }

// The search of a wave whose particles are all interior (FAST): per stencil column the union of
// the 64 lanes' candidate ranges is one short index range (the lanes are consecutive in cell
// order, mostly inside one or two cell columns), so the wave stages it in LDS with coalesced
// loads and every lane then tests its own candidates from LDS.  The global gathers of the
// per-lane loop cost ~19 L1 tag lookups per load instruction (PMC, profiles/r01) and the
// texture-address unit was the bound; a staged column costs 4.  Same candidates, same order and,
// where it decides, the same FP64 test as scan_candidates, so the list is identical.  Every lane of
// the wave must call this (act = live particle); the column loop and the staging are wave-uniform.
//
// Per column the wave waits for memory once: the start[] loads of column col + 1 are issued before
// column col's staging loads, so the one wait for the staging also covers them and the next
// column's window is ready at once.  hipcc would wait for them at their first use instead (round 3:
// predicated loads, a register copy at the loop latch, a merge with the list stores pending on
// the same counter -- each made it emit vmcnt(0) right after issuing them: two round trips per
// column), so they are issued in asm (start_load), which hipcc does not count, and every path of a
// column ends in an explicit vmcnt(0) before the next column reads them (start_landed).
template <int DIM, int PERM, int SB = MPH_SB, int CAP = MPH_LDS_CAP>
__device__ __forceinline__ int scan_candidates_lds(const DevParams& P, const Soa& A, const int* start,
                                                   int i, bool act, double xi, double yi, double zi,
                                                   int cx, int cy, int cz, int* out, double* sx, int* stored,
                                                   unsigned long long* lgap, unsigned long long* lhdr)
{
    // the staging area holds the window's 16-byte FP32 records, SB past the window's end
    constexpr int kCap32 = stage_words(CAP, SB) / 2 - SB - 1;
    const int lane = threadIdx.x & 63;
    // buffer descriptor of the wave's ELL tile (out - lane, wave-uniform): list stores take a 32-bit
    // lane offset instead of a 64-bit address; a store past the tile is dropped by the hardware
    const unsigned long long tb = (unsigned long long)(out - lane);
    const unsigned tlo = __builtin_amdgcn_readfirstlane((unsigned)tb);
    const unsigned thi = __builtin_amdgcn_readfirstlane((unsigned)(tb >> 32));
    const __amdgpu_buffer_rsrc_t tile_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((unsigned long long)thi << 32) | tlo), 0, kTile * kTileRows * (int)sizeof(int),
        0x00020000);
    const double lo2 = P.rc2_lo, hi2 = P.rc2_hi;
    using X = CellAxes<DIM, PERM>;
    constexpr int NCOL = DIM == 3 ? kGroups * kGroups : kGroups;
    const int cc[3] = {cx, cy, cz};
    const int cca = cc[X::A2];
    const double cw0 = P.cwid[X::A0], cw1 = P.cwid[X::A1];
    const double uu[3] = {grid_offset(xi, P.corg[0], P.dw[0]), grid_offset(yi, P.corg[1], P.dw[1]),
                          DIM == 3 ? grid_offset(zi, P.corg[2], P.dw[2]) : 0.0};
    const double ua = uu[X::A2];
    const double ginva = P.ginv[X::A2];
    // Candidate range of this lane in stencil column col (cell ranges -> start[] loads).  The
    // trimming is only a bound (the exact test decides), so it runs in FP32 from per-lane values
    // computed once (the offsets inside the own cell across the columns and along the contiguous
    // axis, the row base), every rounding outwards by an absolute margin: the squared cell gaps
    // down (2^-20 cell widths), the cutoff and the half range up, the range ends out by 1e-3
    // cells.  Each range therefore holds the FP64 one (a superset: same candidates, same list).
    // The contiguous-axis offset is taken relative to the own cell in FP64 before the conversion
    // (ua ginv - c lies in [0, 1) for an interior lane), so the margin holds on any grid size.
    // The gap along the slowest axis changes once per group of columns (visited in order).
    // An inactive lane gets a negative cutoff (no column opens); the gap margin mu is folded into
    // the subtracted offsets; the range ends carry a bias of kBias cells, so truncation is floor
    // (the ends lie within a few cells of the own cell) and the bias comes off in the row base.
    // Each added rounding is below 1e-5 cells or 2^-24 of a cell width, far inside the margins.
    constexpr float kDn = 1.0f - 1.0f / (1 << 20), kUp = 1.0f + 1.0f / (1 << 19);
    constexpr float kBias = 32.0f;
    const float rcm2f = act ? (float)P.rc2_trim * kUp : -1.0f;
    float gx2f = 0.0f;
    const int c0l = cc[X::A0], c1l = DIM == 3 ? cc[X::A1] : 0;
    const float cw0f = (float)cw0, cw1f = (float)cw1;
    const float f0 = (float)(uu[X::A0] - c0l * cw0), f1 = DIM == 3 ? (float)(uu[X::A1] - c1l * cw1) : 0.0f;
    const float mu0 = cw0f * (1.0f / (1 << 20)), mu1 = cw1f * (1.0f / (1 << 20));
    const float g0p = f0 + mu0, g0m = (cw0f - f0) + mu0, g1p = f1 + mu1, g1m = (cw1f - f1) + mu1;
    const float ginvaf = (float)ginva;
    const float caf = (float)(ua * ginva - (double)cca);   // offset inside the own cell, cells
    const float cal = (caf - 1e-3f) + kBias, cah = (caf + 1e-3f) + kBias;
    const float rgf = kUp * ginvaf;
    const int rowbase = (DIM == 3 ? (c0l * P.gc[X::A1] + c1l) * P.gc[X::A2] : c0l * P.gc[1]) + cca - (int)kBias;
    const int sa = P.sa;
    const __amdgpu_buffer_rsrc_t srs = arr_rsrc(start);
    auto gap32 = [](int d, float cwf, float gp, float gm) {
        if (d == 0) return 0.0f;
        const float v = (float)(d > 0 ? d : -d) * cwf - (d > 0 ? gp : gm);
        return v > 0.0f ? v : 0.0f;
    };
    auto col_range = [&](int col, int& jb, int& je) {
        int cofs;
        float d2f;
        if (DIM == 3) {
            const int dxc = col / kGroups - kReach, dyc = col % kGroups - kReach;
            if (dyc == -kReach) {
                const float gx = gap32(dxc, cw0f, g0p, g0m);
                gx2f = gx * gx * kDn;
            }
            const float gy = gap32(dyc, cw1f, g1p, g1m);
            d2f = (gx2f + gy * gy * kDn) * kDn;
            cofs = (dxc * P.gc[X::A1] + dyc) * P.gc[X::A2];
        } else {
            const int dxc = col - kReach;
            const float gx = gap32(dxc, cw0f, g0p, g0m);
            d2f = gx * gx * kDn;
            cofs = dxc * P.gc[1];
        }
        const bool ok = d2f <= rcm2f;
        const float rc = __builtin_amdgcn_sqrtf(fmaxf(rcm2f - d2f, 0.0f)) * rgf;   // half range, cells
        const int lo = max((int)(cal - rc), (int)kBias - sa);
        const int hi = min((int)(cah + rc), (int)kBias + sa);
        const int b = rowbase + cofs;
        // a lane without candidates reads start[0] twice (empty range)
        start_load2(srs, ok ? (unsigned)(b + lo) * 4u : 0u, ok ? (unsigned)(b + hi + 1) * 4u : 0u, jb, je);
    };
    // the lane's next list slot: soff = stored * 256 + lane * 4 (one add per entry, no address
    // arithmetic); bits 18 and up count every accepted neighbour (NeighborCount), bits 8-17 the
    // stored ones (the FP32 path keeps only r^2 <= P.rlf: kListTotal, kListKeep), so the store
    // offset is soff & kSoffMask
    int soff = lane << 2;
    // Row jumps (aligned rows, see RowMask): at the end of a stencil group (3-D: the 7 columns of
    // one slowest-axis offset; 2-D: a column) the lanes' next rows move on to the wave's highest
    // row, so the next group's entries start on one row for all lanes however far their counts
    // drifted (off the lattice a store instruction otherwise touches as many rows as it has lanes,
    // and the list lines leave L2 partly written).  Only while the highest
    // row is below kAlignRows and the rows differ by kAlignDrift or more; on the lattice the lanes'
    // counts agree and the wave keeps plain rows.
    // The jumps are recorded as they happen (byte stores: the wave's header byte k, the lane's gap
    // byte k), so that no register holds them across the columns (the search is at its 64-VGPR
    // budget); the jump count goes to header byte 7 at the end.
    // jumps: the jumps so far, plus kMaxJumps + 1 once the wave stops jumping (one SGPR)
    constexpr int GSZ = DIM == 3 ? kGroups : 1;
    // (3-D only: the 2-D lists, ~20 entries in 7 columns, drift little, and the checks cost the Bar
    // search 9 %)
    int jumps = DIM == 3 && kAlignDrift <= kAlignRows ? 0 : kMaxJumps + 1;   // (stopped, none made)
    // the wave's header bytes, formed where they are stored (not held in SGPRs across the columns)
    auto hdr_byte = [&](int k) {
        int ii = i;
        asm volatile("" : "+v"(ii));
        return reinterpret_cast<unsigned char*>(lhdr + __builtin_amdgcn_readfirstlane(ii >> 6)) + k;
    };
    auto group_end = [&]() {
        if (jumps >= kMaxJumps) return;
        const int row = soff_stored(soff);
        const int m = __builtin_amdgcn_readfirstlane(wave_max(row));
        if (m >= kAlignRows) {
            jumps += kMaxJumps + 1;   // no more jumps
            return;
        }
        if (kAlignDrift <= 1) {
            if (!__ballot(act && row != m)) return;   // the rows agree
        } else {
            const int mn = __builtin_amdgcn_readfirstlane(wave_min(act ? row : m));
            if (m - mn < kAlignDrift) return;
        }
        // the address formed here, not hoisted out of the column loop as a register pair
        int ii = i;
        asm volatile("" : "+v"(ii));
        reinterpret_cast<unsigned char*>(lgap + ii)[jumps] = (unsigned char)row;   // the lane's gap [row, m)
        if (lane == 0) *hdr_byte(jumps) = (unsigned char)m;
        soff += (m - row) << 8;
        ++jumps;
    };
    constexpr int kSelfCol = DIM == 3 ? kReach * kGroups + kReach : kReach;   // the lane's own column
    // one stencil column: its range [jb, je) was loaded one column ahead; (nb_jb, nb_je) receive
    // column col + 1's.  The loop below is unrolled by two with the roles of the two register pairs
    // swapped, so no copy at the loop latch waits for the loads in flight.
    auto column = [&](int col, int jb, int je, int& nb_jb, int& nb_je) {
        start_landed(jb, je);   // loaded one column ahead; every path below ended in vmcnt(0)
        if (col > 0 && col % GSZ == 0) group_end();
        if (col + 1 < NCOL) col_range(col + 1, nb_jb, nb_je);
        const bool any = je > jb;
        // the wave's window [mn, mx): the lanes are in cell order, so the first lane with candidates
        // normally has the lowest jb and the last the highest je -- read those two lanes, and take
        // the DPP reductions only when a lane says otherwise (wave-uniform check)
        const unsigned long long am = __ballot(any);
        if (!am) {   // wave-uniform: no lane has candidates in this column
            // wait here for column col + 1's start[] loads, so that every path into the next column
            // has them landed and its first use needs no wait (which would also wait for this
            // column's list stores: loads and stores share vmcnt)
            __builtin_amdgcn_s_waitcnt(0x0F70);
            return;
        }
        int mn = __builtin_amdgcn_readlane(jb, __ffsll((long long)am) - 1);
        int mx = __builtin_amdgcn_readlane(je, 63 - __clzll(am));
        if (__ballot(any && (jb < mn || je > mx))) {
            mn = wave_min(any ? jb : 0x7fffffff);
            mx = wave_max(any ? je : -1);
        }
        const int span = mx - mn;
        // A window wider than the staging area is mostly a wave across two cell rows: its lanes' ranges
        // form two runs far apart.  Split the lanes at the widest gap (a lane whose range starts past
        // every earlier lane's end) and stage each run's window, one after the other, when both fit.
        int lbase = mn, n1 = span, m2 = 0, n2 = 0;   // lane's record index j - lbase; the two windows
        bool two = false;
        if (span > kCap32) {   // wave-uniform, rare
            int pm = any ? je : -1;   // running max of the ends over the lanes below and at this one
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(pm, o, 64);
                if (lane >= o) pm = max(pm, v);
            }
            int ex = __shfl_up(pm, 1, 64);
            if (lane == 0) ex = -1;
            const int gap = any && ex >= 0 ? jb - ex : -1;
            const int gmax = wave_max(gap);
            if (gmax > 0) {
                const int sl = __ffsll((long long)__ballot(gap == gmax)) - 1;
                const bool hi_run = lane >= sl;
                const int m1 = wave_min(any && !hi_run ? jb : 0x7fffffff);
                const int x1 = __builtin_amdgcn_readlane(ex, sl);   // the low run's end
                m2 = wave_min(any && hi_run ? jb : 0x7fffffff);
                n1 = x1 - m1;
                n2 = mx - m2;
                if (n1 + n2 <= kCap32) {
                    two = true;
                    lbase = hi_run ? m2 - n1 : m1;
                    mn = m1;
                }
            }
        }
        if (span <= kCap32 || two) {
            // FP32 records: candidate j at record j - lbase, 64 records (1 KB) per instruction
            float4* s4 = reinterpret_cast<float4*>(sx);
            for (int p = 0; p * 64 < n1; ++p)   // wave-uniform
                if (p * 64 + lane < n1) __builtin_amdgcn_global_load_lds(A.f4 + mn + p * 64 + lane, s4 + p * 64, 16, 0, 0);
            for (int p = 0; p * 64 < n2; ++p)   // the second run (two), after the first
                if (p * 64 + lane < n2)
                    __builtin_amdgcn_global_load_lds(A.f4 + m2 + p * 64 + lane, s4 + n1 + p * 64, 16, 0, 0);
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the records (and column col + 1's start[]) landed
            __builtin_amdgcn_wave_barrier();
            const float xf = (float)(xi - P.cref[0]), yf = (float)(yi - P.cref[1]), zf = (float)(zi - P.cref[2]);
            const float lof = P.rc2f_lo, hif = P.rc2f_hi;
            auto test32 = [&](auto self_tag) {
                constexpr bool SELF = decltype(self_tag)::value;
                for (int j0 = jb; j0 < je; j0 += SB) {
                    float4 r[SB];
#pragma unroll
                    for (int u = 0; u < SB; ++u) r[u] = s4[j0 - lbase + u];
#pragma unroll
                    for (int u = 0; u < SB; ++u) {
                        const int j = j0 + u;
                        const float dx = r[u].x - xf, dy = r[u].y - yf, dz = r[u].z - zf;
                        const float r2f = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
                        bool live = true;
                        if (u > 0) live = j < je;
                        if (SELF) live = live & (j != i);
                        // two compares; the band as wave masks (SALU), its lane bit read only inside
                        // the rare branch
                        const bool le_lo = r2f <= lof, le_hi = r2f <= hif;
                        bool a = live & le_lo;
                        const unsigned long long mband = __builtin_amdgcn_ballot_w64(le_hi) &
                                                         ~__builtin_amdgcn_ballot_w64(le_lo) &
                                                         __builtin_amdgcn_ballot_w64(live);
                        if (mband) {   // rare (wave-uniform): the FP64 test on the global positions
                            // the band lanes straight from the mask (no per-lane compare)
                            if (__builtin_amdgcn_inverse_ballot_w64(mband)) {
                                // the index hidden from the loop's induction analysis, so the addresses
                                // are formed here and not carried through the loop
                                int jj = j;
                                asm volatile("" : "+v"(jj));
                                const double ddx = A.x[jj] - xi, ddy = A.y[jj] - yi, ddz = A.z[jj] - zi;
                                const double r2a = fma(ddx, ddx, fma(ddy, ddy, ddz * ddz));
                                const bool in = r2a <= lo2;
                                a = in;
                                if ((r2a <= hi2) != in) a = accept_band(P, ddx, ddy, ddz);
                            }
                        }
                        if (a) {
                            // stored when within the passes' largest radius (FP32, an upper bound:
                            // the passes' own exact tests decide); counted always
                            const bool keep = r2f <= P.rlf;
                            if (keep)
                                __builtin_amdgcn_raw_buffer_store_b32(nbr_entry(j, __float_as_int(r[u].w)), tile_rsrc,
                                                                      soff & kSoffMask, 0, 0);
                            soff += keep ? kListKeep : kListTotal;
                        }
                    }
                }
            };
            if (col == kSelfCol) test32(std::true_type{});
            else test32(std::false_type{});
            __builtin_amdgcn_wave_barrier();   // every lane done reading before the next staging
        } else {
            // a window wider than the staging area: per-lane gathers, every accepted pair stored
            for (int j0 = jb; j0 < je; j0 += SB) {
                double xs[SB], ys[SB], zs[SB];
#pragma unroll
                for (int u = 0; u < SB; ++u) {
                    const int j = j0 + u < je ? j0 + u : je - 1;
                    xs[u] = A.x[j];
                    ys[u] = A.y[j];
                    zs[u] = A.z[j];
                }
#pragma unroll
                for (int u = 0; u < SB; ++u) {
                    const int j = j0 + u;
                    if (accept_interior(P, xs[u] - xi, ys[u] - yi, zs[u] - zi, lo2, hi2) && j < je && j != i) {
                        const int row = soff_stored(soff);
                        if (soff_total(soff) < kMaxNeighbor && row < kTileRows)
                            out[(size_t)row * kTile] = nbr_entry(j, A.type[j]);
                        soff += kListKeep;
                    }
                }
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);   // column col + 1's start[] loads (wide windows are rare)
        }
    };
    int ra_b, ra_e, rb_b = 0, rb_e = 0;   // the two register pairs of the column ranges
    col_range(0, ra_b, ra_e);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    for (int col = 0; col < NCOL; col += 2) {
        column(col, ra_b, ra_e, rb_b, rb_e);
        if (col + 1 < NCOL) column(col + 1, rb_b, rb_e, ra_b, ra_e);
    }
    *stored = soff_stored(soff);  // the list's rows, gaps included (entries: r^2 <= P.rlf)
    if (lane == 0) *hdr_byte(7) = (unsigned char)(jumps > kMaxJumps ? jumps - kMaxJumps - 1 : jumps);
    return soff_total(soff);      // every neighbour (NeighborCount)
}

// Slab mode: true when no lane of the wave holds an owned particle (ghost ids are negative).
// With the (z, x, y) cell order of z slabs (DevParams.perm) the ghosts beyond the two faces fill
// whole wavefronts at the ends of the sorted arrays; their lists and pass-A/pass-B sums are not
// needed (their pass-A values arrive in the halo, their pass-B results are dropped), so the list
// kernels skip them.
__device__ __forceinline__ bool wave_all_ghosts(const DevParams& P, const Soa& A, bool live, int ii)
{
    if (P.slab_axis < 0) return false;
    return __all(!live || A.id[ii] < 0);
}

// Slab mode: wface[w] = 1 when wave w holds an owned particle within slab_h of a slab face (pass B
// runs it after the halo, phase 2, and the early send takes its particles), else 0 (interior
// waves and waves of ghosts only, phase 1).  Written by the search, so that each pass-B launch
// drops the other's waves with one load; the redistribution of the next step reads it too.
__device__ __forceinline__ void slab_wave_flag(const DevParams& P, const Soa& A, int i, int n, int* wface)
{
    if (P.slab_axis < 0 || !wface) return;
    const bool live = i < n;
    const int ii = live ? i : n - 1;
    const bool own = live && A.id[ii] >= 0;
    const double c = P.slab_axis == 0 ? A.x[ii] : (P.slab_axis == 1 ? A.y[ii] : A.z[ii]);
    const bool inner = c - P.slab_lo > P.slab_h && P.slab_hi - c > P.slab_h;
    const bool face = !__all(!own || inner);
    if ((threadIdx.x & 63) == 0) wface[i >> 6] = face ? 1 : 0;
}

// ncount: the rows of each particle's stored list, gaps included (what the passes walk; the
// entries, r^2 <= P.rlf, are the rows outside the gaps, RowMask); nbcount: NeighborCount, every
// neighbour within the search radius; lhdr / lgap: the row jumps (RowMask)
template <int DIM, int PERM>
__device__ __forceinline__ int neighbors_body(const DevParams& P, const Soa& A, const int* start, int* nbr,
                                               int* ncount, int* nbcount, unsigned long long* lhdr,
                                               unsigned long long* lgap, DevState* st, double* stage, int i)
{
    const int n = dev_n(P);
    const bool live = i < n;
    const int ii = live ? i : n - 1;
    const int tile = __builtin_amdgcn_readfirstlane(i >> 6);
    // a wave past the last particle (the launch has whole blocks of 4 waves): nothing to do, and its
    // tile lies past the list array (sized for the particles' tiles)
    if (tile * kTile >= n) return 0;
    if (wave_all_ghosts(P, A, live, ii)) {
        if (live) ncount[i] = 0;
        if (live) nbcount[i] = 0;
        if ((threadIdx.x & 63) == 0) lhdr[tile] = 0;
        return 0;
    }
    // the ghost lanes of a mixed wave take no part either (empty list)
    const bool own = live && !(P.slab_axis >= 0 && A.id[ii] < 0);
    const double xi = A.x[ii], yi = A.y[ii], zi = A.z[ii];
    const bool fast = wave_search_interior(P, st, own, xi, yi, zi);
    int cnt = 0, stored = 0;
    const int cx = cell_axis(xi, P.corg[0], P.dw[0], P.ginv[0], P.gc[0]);
    const int cy = cell_axis(yi, P.corg[1], P.dw[1], P.ginv[1], P.gc[1]);
    const int cz = DIM == 3 ? cell_axis(zi, P.corg[2], P.dw[2], P.ginv[2], P.gc[2]) : 0;
    int* out = nbr + (size_t)(i >> 6) * kTileStride + (i & 63);
    if (fast) {
        cnt = scan_candidates_lds<DIM, PERM>(P, A, start, i, own, xi, yi, zi, cx, cy, cz, out, stage, &stored,
                                             lgap, lhdr);
    } else {
        if (own)
            cnt = scan_candidates<DIM, false, PERM>(P, A, start, i, xi, yi, zi, cx, cy, cz, out);
        stored = cnt;
        if ((threadIdx.x & 63) == 0) lhdr[tile] = 0;   // plain rows
    }
    if (live) ncount[i] = stored;
    if (live) nbcount[i] = cnt;
    // overflow flag (main.cpp:1766-1768 is the reference's limit).  No per-step statistics here:
    // one same-address device atomic per wave serialises at ~11 ns each (21.8k waves at D1M took
    // 0.5 ms); mph_neighbor_stats reduces ncount on demand.
    if (cnt > kMaxNeighbor) atomicOr(&st->overflow, 1);
    return stored;
}

// one kernel per cell order (DevParams.perm), so each keeps its own register budget; held to 64
// VGPRs (8 waves per SIMD: the search waits on its start[] and staging loads).  bal: the passes'
// XCD split runs (launch_sort), so the waves feed its histogram.
#ifndef MPH_NB_WPE
#define MPH_NB_WPE 8
#endif
template <int DIM, int PERM>
__global__ __launch_bounds__(MPH_LB) __attribute__((amdgpu_waves_per_eu(MPH_NB_WPE))) void k_neighbors(
    DevParams P, Soa A, const int* __restrict__ start, int* __restrict__ nbr, int* __restrict__ ncount,
    int* __restrict__ nbcount, unsigned long long* __restrict__ lhdr, unsigned long long* __restrict__ lgap,
    DevState* __restrict__ st, int* __restrict__ wface, int bal)
{
    const int n = dev_n(P);
    if ((int)blockIdx.x >= list_blocks(n)) return;
    const int tb = xcd_block(blockIdx.x, list_blocks(n));
    __shared__ __attribute__((aligned(16))) double stage[kWB][stage_words(MPH_LDS_CAP, MPH_SB)];
    const int i = tb * blockDim.x + threadIdx.x;
    slab_wave_flag(P, A, i, n, wface);
    const int cnt = neighbors_body<DIM, PERM>(P, A, start, nbr, ncount, nbcount, lhdr, lgap, st,
                                              stage[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)], i);
    if (bal) add_wave_work(st, cnt, i, n);
}

// ---------------------------------------------------------------------------- pass A -------

// List pass: the neighbour loops gather U neighbours' fields
// before the first use (all loads in flight at once; the loops are memory-latency bound).
#ifndef MPH_UA
#define MPH_UA 5   // pass A (with MPH_PA_WPE 4; coherent gathers at kReach 3: 0.355 ms against 0.376 at U = 8, 3 waves)
#endif
#ifndef MPH_UB
#define MPH_UB 8
#endif
// The rows of a lane's list (RowMask): the lane walks rows [0, end); a row that holds no entry of
// it (a gap of its row jumps, or past its end) gathers nothing and is not summed.
// The batch of U rows from k0: the entries' loads first, then which rows hold entries (bits_of(),
// from the lane's mask in LDS or registers) -- so the loads are in flight while the bits are formed
template <int U, typename Bits>
__device__ __forceinline__ void list_batch(const NbrList& NL, Bits bits_of, int k0, int end,
                                           bool (&ok)[U], int (&jj)[U], int (&TT)[U])
{
    int e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) nbr_at(NL, k0 + u < end ? k0 + u : end - 1, e[u], TT[u]);
    const unsigned bits = bits_of();
#pragma unroll
    for (int u = 0; u < U; ++u) {
        ok[u] = (bits & (1u << u)) != 0;
        jj[u] = e[u];
    }
}

template <bool FAST, int DIM, bool EQR, int U = MPH_UA>
__device__ __forceinline__ void pass_a_loop(const DevParams& P, const double* s_ratio, const double* s_mu,
                                            const Soa& A,
                                            NbrList NL, bool plain, const unsigned* lm, int end, int ti,
                                            bool solid, double xi, double yi, double zi, double vxi, double vyi,
                                            double vzi, PassA& o)
{
    const __amdgpu_buffer_rsrc_t p6r = sized_rsrc(A.p6, (unsigned)P.n * 48u);
    for (int k0 = 0; k0 < end; k0 += U) {
        int jj[U];
        double X[U], Y[U], Z[U], VX[U], VY[U], VZ[U];
        int TT[U];
        bool ok[U];
        list_batch<U>(NL, [&] { return plain ? bit_range(0, end - k0) : row_bits_lds(lm, k0, end); }, k0, end,
                      ok, jj, TT);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // a row without an entry of the lane (a gap, or past its end) reads past the buffer:
            // zeros, no cache lookup
            const unsigned off = ok[u] ? (unsigned)jj[u] * 48u : kGatherOob;
            const double2 a = buf_ld16(p6r, off), b = buf_ld16(p6r, off + 16u), c = buf_ld16(p6r, off + 32u);
            X[u] = a.x; Y[u] = a.y; Z[u] = b.x;
            VX[u] = b.y; VY[u] = c.x; VZ[u] = c.y;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // the gathered values used on every path, so that hipcc does not sink a row's loads into
            // its `ok` branch (issued there, late, they would not overlap the batch's other loads)
            asm volatile("" ::"v"(X[u]), "v"(Y[u]), "v"(Z[u]), "v"(VX[u]), "v"(VY[u]), "v"(VZ[u]));
            if (!ok[u]) continue;
            const double q0 = image_exact<FAST>(X[u] - xi, P.dw[0], P.hw[0], P.w075[0]);
            const double q1 = image_exact<FAST>(Y[u] - yi, P.dw[1], P.hw[1], P.w075[1]);
            const double q2 = image_exact<FAST || DIM == 2>(Z[u] - zi, P.dw[2], P.hw[2], P.w075[2]);
            pass_a_term<true, EQR>(P, s_ratio, s_mu, ti, TT[u], solid, q0, q1, q2, r2_exact(q0, q1, q2),
                                   VX[u] - vxi, VY[u] - vyi, VZ[u] - vzi, o);
        }
    }
}

#ifndef MPH_PA_WPE
#define MPH_PA_WPE 4   // pass A at <= 128 VGPRs: 4 waves per SIMD
#endif
#if MPH_PA_WPE
#define MPH_PA_ATTR __attribute__((amdgpu_waves_per_eu(MPH_PA_WPE)))
#else
#define MPH_PA_ATTR
#endif
template <int DIM>
__global__ __launch_bounds__(MPH_LB) MPH_PA_ATTR void k_pass_a(DevParams P, const DevTables* __restrict__ T, Soa A,
                                                const int* __restrict__ nbr,
                                                const int* __restrict__ ncount,
                                                const unsigned long long* __restrict__ lhdr,
                                                const unsigned long long* __restrict__ lgap, PassAOut pout,
                                                const DevState* __restrict__ st)
{
    const int n = dev_n(P);
    const int lb = list_block(st, n, MPH_PASS_A_REV);
    if (lb < 0) return;
    __shared__ double s_ratio[kTypes * kTypes];
    __shared__ double s_mu[kTypes * kTypes];
    if (threadIdx.x < kTypes * kTypes) {
        s_ratio[threadIdx.x] = T->ratio[threadIdx.x];
        s_mu[threadIdx.x] = T->mu_ij[threadIdx.x] * (-P.cvis * P.cdv * P.vol);   // pass_a_term's viscous factor
    }
    __syncthreads();
    const int i = lb * blockDim.x + threadIdx.x;
    const bool live = i < n;
    const int ii = live ? i : n - 1;
    const double xi = A.x[ii], yi = A.y[ii], zi = A.z[ii];
    if (wave_all_ghosts(P, A, live, ii)) {
        // ghosts: PressureP (+ GravityCenter, PressureA) arrive in the halo, which also fills the
        // .w of the pass-B record; its position part is written here
        if (live && pout.rec) rec_store(pout.rec, P.n, i, xi, yi, zi, 0.0);
        return;
    }
    // likewise the ghost lanes of a mixed wave
    const bool ghost = live && P.slab_axis >= 0 && A.id[ii] < 0;
    if (ghost && pout.rec) rec_store(pout.rec, P.n, i, xi, yi, zi, 0.0);
    const bool own = live && !ghost;
    // the search's rule (its list order and the fast minimum image go together)
    const bool fast = wave_search_interior(P, st, own, xi, yi, zi);
    if (!own) return;
    double vxi, vyi, vzi;
    own_velocity(A, i, vxi, vyi, vzi);
    const int ti = A.type[i];
    const bool solid = dev_is_struct(ti);
    const int end = ncount[i] < kTileRows ? ncount[i] : kTileRows;
    __shared__ unsigned s_mask[kWB][kTile * kMaskWords];
    unsigned* lm = &s_mask[threadIdx.x >> 6][(threadIdx.x & 63) * kMaskWords];
    // a wave without jumps (plain rows: on the lattice, in 2-D) needs no mask, only its lanes' ends
    const unsigned long long hdr = wave_hdr(lhdr, i);
    const bool plain = (hdr >> 56) == 0;
    if (!plain) mask_to_lds(lm, row_mask(hdr, lgap, i, end));   // (each lane reads back only its own)
    const NbrList NL = nbr_list(nbr, i);
    PassA o;
    // wave-uniform: equal radii (every BASELINE config) take the single-cutoff form of the sums in
    // the interior waves; waves at a periodic face keep the general form
    const bool eqr = pass_a_equal_radii(P);
    if (fast && eqr)
        pass_a_loop<true, DIM, true>(P, s_ratio, s_mu, A, NL, plain, lm, end, ti, solid, xi, yi, zi, vxi, vyi, vzi, o);
    else if (fast)
        pass_a_loop<true, DIM, false>(P, s_ratio, s_mu, A, NL, plain, lm, end, ti, solid, xi, yi, zi, vxi, vyi, vzi, o);
    else
        pass_a_loop<false, DIM, false>(P, s_ratio, s_mu, A, NL, plain, lm, end, ti, solid, xi, yi, zi, vxi, vyi, vzi, o);
    pass_a_finish(P, T, ti, i, o, pout, xi, yi, zi);
}

// Displacement u = Mod(x - x0 + W/2, W) - W/2 of calculateElasticDeformationVector (2700-2712),
// computed once per slot and substep instead of once per pair (same expression, same bits).
__device__ __forceinline__ double4 struct_disp(const DevParams& P, double4 x, double4 x0)
{
    return make_double4(image_exact<false>(x.x - x0.x, P.dw[0], P.hw[0], P.w075[0]),
                        image_exact<false>(x.y - x0.y, P.dw[1], P.hw[1], P.w075[1]),
                        image_exact<false>(x.z - x0.z, P.dw[2], P.hw[2], P.w075[2]), 0.0);
}

// ---------------------------------------------------------------------------- pass B -------

// Pass B needs, per neighbour, only what pass A could not know: P_j (and, with surface tension,
// GC_j and PA_j).  The P_i half of the pressure force and the viscous force were summed in pass A
// (fpart), so the gather per neighbour is one 32-byte record {x, y, z, P} (two 16-byte planes,
// rec_load); the type of j (in the list entry) only for structure i (InterfaceForce) or surface
// tension.
// One neighbour's pair forces for pass B (see k_pass_b): PressureP's P_j half, and with surface
// tension PressureA and DiffuseInterface; structure i takes non-structure j only.
template <bool FAST, bool SURF, int DIM>
__device__ __forceinline__ void pass_b_term(const DevParams& P, const double* s_ratio, const double* gx,
                                            const double* gy, const double* gz, const double* pa, int j, int tj,
                                            double X, double Y, double Z, double PJ, int ti, bool solid,
                                            double xi, double yi, double zi, double gxi, double gyi, double gzi,
                                            double pai, double ai, double dscale, double cpv, double& f0,
                                            double& f1, double& f2)
{
    if (solid && dev_is_struct(tj)) return;
    const double q0 = image_exact<FAST>(X - xi, P.dw[0], P.hw[0], P.w075[0]);
    const double q1 = image_exact<FAST>(Y - yi, P.dw[1], P.hw[1], P.w075[1]);
    const double q2 = image_exact<FAST || DIM == 2>(Z - zi, P.dw[2], P.hw[2], P.w075[2]);
    const double r2 = r2_exact(q0, q1, q2);
    if (!SURF || solid) {
        if (r2 < P.rp2) {
            double r, ir;
            rsqrt_pair(r2, r, ir);
            // dw_p(r) / r = cdp (1 - r / rp) / r = cdp (1/r - 1/rp): r itself is not needed
            const double c = PJ * cpv * (ir - P.inv_rp);
            f0 += c * q0;
            f1 += c * q1;
            f2 += c * q2;
        }
        return;
    }
    double r, ir;
    rsqrt_pair(r2, r, ir);
    double c = 0.0;
    if (r2 < P.rp2) c += PJ * (cpv * (1.0 - r * P.inv_rp)) * ir;
    const double rij = s_ratio[ti * kTypes + tj];
    const double rji = s_ratio[tj * kTypes + ti];
    const double gxj = gx[j], gyj = gy[j], gzj = gz[j], paj = pa[j];
    if (r2 < P.ra2) {
        const double t = r * P.inv_ra;
        const double dwa = P.cda * (1.0 - t) * (1.0 - 3.0 * t);
        c += (pai * rij + paj * rji) * dwa * ir * P.vol;
    }
    if (r2 < P.rg2) {
        const double omt = 1.0 - r * P.inv_rg;
        const double wg = P.cg * omt * omt;
        const double dwg = P.cdg * omt;
        const double wij = rij * wg, wji = rji * wg;
        f0 -= (ai * gxj * wji - ai * gxi * wij) * dscale;
        f1 -= (ai * gyj * wji - ai * gyi * wij) * dscale;
        f2 -= (ai * gzj * wji - ai * gzi * wij) * dscale;
        const double dwij = rij * dwg, dwji = rji * dwg;
        const double gr = (ai * gxj * dwji - ai * gxi * dwij) * q0 +
                          (ai * gyj * dwji - ai * gyi * dwij) * q1 +
                          (ai * gzj * dwji - ai * gzi * dwij) * q2;
        c -= gr * ir * dscale;
    }
    f0 += c * q0;
    f1 += c * q1;
    f2 += c * q2;
}

template <bool FAST, bool SURF, int DIM, int U = MPH_UB>
__device__ __forceinline__ void pass_b_loop(const DevParams& P, const double* s_ratio,
                                            const double4* rec, const double* gx,
                                            const double* gy, const double* gz, const double* pa,
                                            NbrList NL, bool plain, const RowMask& M, int end, int ti, bool solid,
                                            double xi, double yi, double zi, double gxi, double gyi, double gzi,
                                            double pai, double ai, double& f0, double& f1, double& f2)
{
    const double dscale = P.rg_r2g * (P.vol / P.dx);
    const double cpv = P.cdp * P.vol;
    // the record's two planes {x, y} at [j], {z, P} at [ps + j] (rec_load), 16 bytes each
    const unsigned ps16 = (unsigned)P.n * 16u;
    const __amdgpu_buffer_rsrc_t recr = sized_rsrc(rec, 2u * ps16);
    for (int k0 = 0; k0 < end; k0 += U) {
        int jj[U];
        double X[U], Y[U], Z[U], PJ[U];
        int TT[U];
        bool ok[U];
        list_batch<U>(NL, [&] { return plain ? bit_range(0, end - k0) : row_bits(M, k0, end); }, k0, end, ok, jj,
                      TT);
#pragma unroll
        for (int u = 0; u < U; ++u) {   // (rows without an entry: past the buffer, as in pass_a_loop)
            const unsigned off = ok[u] ? (unsigned)jj[u] * 16u : kGatherOob;
            const double2 a = buf_ld16(recr, off), b = buf_ld16(recr, off == kGatherOob ? off : off + ps16);
            X[u] = a.x; Y[u] = a.y; Z[u] = b.x; PJ[u] = b.y;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            asm volatile("" ::"v"(X[u]), "v"(Y[u]), "v"(Z[u]), "v"(PJ[u]));   // (see pass_a_loop)
            if (!ok[u]) continue;
            pass_b_term<FAST, SURF, DIM>(P, s_ratio, gx, gy, gz, pa, jj[u], TT[u], X[u], Y[u], Z[u], PJ[u], ti,
                                         solid, xi, yi, zi, gxi, gyi, gzi, pai, ai, dscale, cpv, f0, f1, f2);
        }
    }
}

// Pair forces of PressureP (2394-2424), PressureA (2225-2258), DiffuseInterface (2261-2312),
// ViscosityV (2478-2522) for non-structure i; InterfaceForce (2439-2472) for structure i; then
// Gravity (2917-2936), Acceleration/kick (2938-2956) and Convection/drift (1892-1907).  The sums
// start from pass A's fpart (P_i half of the pressure force + viscous force).
template <bool SURF, int DIM>
#ifndef MPH_PB_WPE
#define MPH_PB_WPE 0   // pass B occupancy hint (0: the compiler's choice, 112 VGPRs / 4 waves at U = 8)
#endif
#if MPH_PB_WPE
#define MPH_PB_ATTR __attribute__((amdgpu_waves_per_eu(MPH_PB_WPE)))
#else
#define MPH_PB_ATTR
#endif
__global__ __launch_bounds__(MPH_LB) MPH_PB_ATTR void k_pass_b(DevParams P, const DevTables* __restrict__ T, Soa A,
                                                const double4* __restrict__ rec,
                                                const double4* __restrict__ fpart,
                                                const double* __restrict__ gx,
                                                const double* __restrict__ gy,
                                                const double* __restrict__ gz,
                                                const double* __restrict__ pa,
                                                const int* __restrict__ nbr,
                                                const int* __restrict__ ncount,
                                                const unsigned long long* __restrict__ lhdr,
                                                const unsigned long long* __restrict__ lgap,
                                                double4* __restrict__ force, double4* __restrict__ acc,
                                                Soa B, int phase, int* __restrict__ wface, StructHook H,
                                                const DevState* __restrict__ st)
{
    const int n = dev_n(P);
    const int lb = list_block(st, n);
    if (lb < 0) return;
    __shared__ double s_ratio[kTypes * kTypes];
    if (SURF) {
        if (threadIdx.x < kTypes * kTypes) s_ratio[threadIdx.x] = T->ratio[threadIdx.x];
        __syncthreads();
    }
    const int i = lb * blockDim.x + threadIdx.x;
    const int ii = i < n ? i : n - 1;
    const double xi = A.x[ii], yi = A.y[ii], zi = A.z[ii];
    bool live = i < n;
    if (phase) {
        // slab mode: phase 1 = the waves without a particle near a face (run while the halo of
        // pass-A values is in flight; also the waves of ghosts only), phase 2 = the rest, after the
        // halo arrived -- split by whole waves (wface, written by the search), so that no wave runs
        // its list loop twice
        const int f = wface[__builtin_amdgcn_readfirstlane(i >> 6)];
        if (phase == 1 ? f != 0 : f == 0) return;
    }
    if (wave_all_ghosts(P, A, live, ii)) {
        if (live) B.id[i] = A.id[i];
        return;
    }
    if (live && P.slab_axis >= 0 && A.id[ii] < 0) {   // a ghost lane of a mixed wave
        B.id[i] = A.id[i];
        live = false;
    }
    const bool fast = wave_search_interior(P, st, live, xi, yi, zi);
    if (!live) return;
    const int ti = A.type[ii];
    const bool solid = dev_is_struct(ti);
    const double4 fp = fpart[ii];
    double f0 = fp.x, f1 = fp.y, f2 = fp.z;
    double gxi = 0.0, gyi = 0.0, gzi = 0.0, pai = 0.0, ai = 0.0;
    if (SURF) {
        gxi = gx[ii]; gyi = gy[ii]; gzi = gz[ii]; pai = pa[ii];
        ai = T->cofa[ti] * P.cofk * P.cofk;
    }
    // a wall's pair forces only go to the Force output (walls are not kicked or drifted, K17/K18):
    // on the steps that do not store it (force null, enqueue_step) its list loop is skipped
    const int end = !force && dev_is_wall(ti) ? 0 : (ncount[i] < kTileRows ? ncount[i] : kTileRows);
    const unsigned long long hdr = wave_hdr(lhdr, i);
    const bool plain = (hdr >> 56) == 0;   // no jumps: rows [0, end) (see k_pass_a)
    const RowMask M = row_mask(hdr, lgap, i, end);
    const NbrList NL = nbr_list(nbr, i);
    if (fast)
        pass_b_loop<true, SURF, DIM>(P, s_ratio, rec, gx, gy, gz, pa, NL, plain, M, end, ti, solid, xi, yi, zi, gxi,
                                     gyi, gzi, pai, ai, f0, f1, f2);
    else
        pass_b_loop<false, SURF, DIM>(P, s_ratio, rec, gx, gy, gz, pa, NL, plain, M, end, ti, solid, xi, yi, zi, gxi,
                                      gyi, gzi, pai, ai, f0, f1, f2);
    double vxi, vyi, vzi;
    own_velocity(A, i, vxi, vyi, vzi);
    double vo0 = vxi, vo1 = vyi, vo2 = vzi;
    double xo0 = xi, xo1 = yi, xo2 = zi;
    double4 ao = make_double4(0.0, 0.0, 0.0, 0.0);
    if (dev_is_fluid(ti) || solid) {
        const double m = T->mass[ti], im = T->inv_mass[ti];
        f0 += m * P.gravity[0];
        f1 += m * P.gravity[1];
        f2 += m * P.gravity[2];
        vo0 += f0 * im * P.dt;
        vo1 += f1 * im * P.dt;
        vo2 += f2 * im * P.dt;
        if (!solid) {
            ao = make_double4(f0 * im, f1 * im, f2 * im, 0.0);
            xo0 += vo0 * P.dt;
            xo1 += vo1 * P.dt;
            xo2 += vo2 * P.dt;
        }
    }
    if (force) {   // null on all but the last step of a replayed batch (enqueue_step)
        force[i] = make_double4(f0, f1, f2, 0.0);
        acc[i] = ao;
    }
    B.x[i] = xo0;
    B.y[i] = xo1;
    B.z[i] = xo2;
    B.vx[i] = vo0;
    B.vy[i] = vo1;
    B.vz[i] = vo2;
    B.type[i] = ti;
    B.id[i] = A.id[i];
    const int id = A.id[i];
    if (solid && H.slot_of && id >= 0) {
        // the elastic substeps' slot-ordered state (structure particles do not drift here);
        // slab mode: slots of owned particles only (ghost ids are negative)
        const int s = H.slot_of[id];
        if (s >= 0) {
            const double4 x4 = make_double4(xo0, xo1, xo2, (double)ti);
            H.sx[s] = x4;
            H.sv[s] = make_double4(vo0, vo1, vo2, 0.0);
            H.su[s] = struct_disp(P, x4, H.sx0[s]);
            H.bidx[s] = i;
        }
    }
}

// ------------------------------------------------------------------------ virial stress ----

// calculateVirialStressAtParticle (main.cpp:3077-3318) for particle i of the current (post-step)
// state: B holds the integrated positions and velocities in A order, the list and the pass-A
// products (PressureP, PressureA, GravityCenter) are this step's.  The reference's four pair
// loops (PressureP 3093-3125, PressureA 3127-3163, viscosity 3165-3206, diffuse interface
// 3208-3282) are one sweep here; every term keeps its own radius test.  All particles, any type.
template <int DIM>
__global__ __launch_bounds__(256) void k_virial(DevParams P, const DevTables* __restrict__ T, Soa A, Soa B,
                                                const double* __restrict__ pres, const double* __restrict__ pa,
                                                const double* __restrict__ gx, const double* __restrict__ gy,
                                                const double* __restrict__ gz, const int* __restrict__ nbr,
                                                const int* __restrict__ ncount,
                                                const unsigned long long* __restrict__ lhdr,
                                                const unsigned long long* __restrict__ lgap,
                                                double* __restrict__ vir, double* __restrict__ vpres)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= dev_n(P)) return;
    if (P.slab_axis >= 0 && A.id[i] < 0) return;   // slab mode: a ghost (its owner computes it)
    const int ti = A.type[i];
    const double xi = B.x[i], yi = B.y[i], zi = B.z[i];
    const double vxi = B.vx[i], vyi = B.vy[i], vzi = B.vz[i];
    const double pi = pres[i], pai = pa[i];
    const double gi[3] = {gx[i], gy[i], gz[i]};
    const double a = T->cofa[ti] * P.cofk * P.cofk;
    const double dscale = P.rg_r2g * (P.vol / P.dx);
    const double cvis = DIM == 2 ? 8.0 : 10.0;
    double S[3][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
    const int end = ncount[i] < kTileRows ? ncount[i] : kTileRows;
    const RowMask M = row_mask(lhdr[i >> 6], lgap, i, end);
    const int* row = ell_row(nbr, i);
    for (int k = 0; k < end; ++k) {
        if (!row_ok(M, k, end)) continue;
        const int e = *ell_at(row, (int)(i & 63), k);
        const int j = e & kIndexMask, tj = e >> kTypeShift;
        double q[3];
        q[0] = image_exact<false>(B.x[j] - xi, P.dw[0], P.hw[0], P.w075[0]);
        q[1] = image_exact<false>(B.y[j] - yi, P.dw[1], P.hw[1], P.w075[1]);
        q[2] = image_exact<DIM == 2>(B.z[j] - zi, P.dw[2], P.hw[2], P.w075[2]);
        const double r2 = r2_exact(q[0], q[1], q[2]);
        if (!(r2 < P.rp2 || r2 < P.ra2 || r2 < P.rv2 || r2 < P.rg2)) continue;
        const double r = sqrt(r2), ir = 1.0 / r;
        const double ratio = T->ratio[ti * kTypes + tj];
        // pair force f_ij = c q_ij + g1 (every term is along q_ij except the first
        // diffuse-interface term); the virial adds f_ij (x) q_ij / V
        double c = 0.0;
        if (r2 < P.rp2) c += pi * (P.cdp * (1.0 - r * P.inv_rp)) * ir * P.vol;          // 3111-3120
        if (r2 < P.ra2) {                                                                // 3147-3156
            const double t = r * P.inv_ra;
            c += pai * (ratio * (P.cda * (1.0 - t) * (1.0 - 3.0 * t))) * ir * P.vol;
        }
        if (r2 < P.rv2) {                                                                // 3183-3199 (x 0.5)
            const double dv = (B.vx[j] - vxi) * q[0] + (B.vy[j] - vyi) * q[1] + (B.vz[j] - vzi) * q[2];
            const double dwij = -(P.cdv * (1.0 - r * P.inv_rv));
            c += 0.5 * (cvis * T->mu_ij[ti * kTypes + tj] * dv * dwij * (ir * ir * ir) * P.vol);
        }
        double g1[3] = {0.0, 0.0, 0.0};
        if (r2 < P.rg2) {                                                                // 3225-3276
            const double omt = 1.0 - r * P.inv_rg;
            const double w = ratio * (P.cg * omt * omt);
            const double dw = ratio * (P.cdg * omt);
            const double gr = -(gi[0] * q[0] + gi[1] * q[1] + gi[2] * q[2]);
            for (int d = 0; d < 3; ++d) g1[d] = a * gi[d] * w * dscale;                 // -a (-GC_i) w
            c += -a * gr * dw * ir * dscale;
        }
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int v = 0; v < 3; ++v) S[u][v] += (c * q[u] + g1[u]) * q[v] / P.vol;
    }
    double* o = vir + (size_t)i * 9;
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int v = 0; v < 3; ++v) o[3 * u + v] = S[u][v];
    vpres[i] = DIM == 2 ? -1.0 / 2.0 * (S[0][0] + S[1][1]) : -1.0 / 3.0 * (S[0][0] + S[1][1] + S[2][2]);
}

// ------------------------------------------------------------------------ elastic solid ----

#ifndef MPH_US
#define MPH_US 4   // batch width of the elastic list loops
#endif

// x0_ij = Mod(x0_j - x0_i + W/2, W) - W/2 and weight(x0_ij, RadiusP) of the fixed Lagrangian
// pair (main.cpp:2705-2716; weight() 268-295, norm over dim components): the same expressions as
// the host's former per-pair table (mph_host.cpp build_structure), recomputed from the 32-byte
// x0 records so that no per-pair table is streamed from HBM every substep.
template <int DIM>
__device__ __forceinline__ double4 struct_pair(const DevParams& P, double4 x0i, double4 x0j)
{
#pragma clang fp contract(off)
    double q[3] = {0.0, 0.0, 0.0};
    q[0] = image_exact<false>(x0j.x - x0i.x, P.dw[0], P.hw[0], P.w075[0]);
    q[1] = image_exact<false>(x0j.y - x0i.y, P.dw[1], P.hw[1], P.w075[1]);
    if (DIM == 3) q[2] = image_exact<false>(x0j.z - x0i.z, P.dw[2], P.hw[2], P.w075[2]);
    double r2 = 0.0;
#pragma unroll
    for (int d = 0; d < DIM; ++d) r2 += q[d] * q[d];
    const double t = sqrt(r2) / P.rp;
    return make_double4(q[0], q[1], q[2], P.cw_pair * ((1.0 - t) * (1.0 - t)));
}

// ELL entry k of slot s (tile width w)
__device__ __forceinline__ size_t sell(int s, int w, int k)
{
    return ((size_t)(s >> 6) * w + k) * 64 + (s & 63);
}

// the G lanes of one structure slot (G | 64, adjacent lanes) sum their strided shares of its list
// in a butterfly: every lane of the group ends with the same total (a + b == b + a exactly)
template <int G>
__device__ __forceinline__ double group_sum(double v)
{
#pragma unroll
    for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o);
    return v;
}

// calculateElasticDeformationVector (2673-2754) + calculateStress (2756-2809) + the first
// Piola-Kirchhoff tensor P = F S L of calculateStressForce (2837-2852).  G lanes per structure
// slot (struct_lanes: enough waves to cover the latency of a small structure), each summing every
// G-th entry of the fixed list, read ELL-tiled in batches of MPH_US; per neighbour only the
// 32-byte displacement record u_j and the x0 record are gathered.
template <int DIM, int G, int U = MPH_US>
__global__ __launch_bounds__(256) void k_struct_stress(DevParams P, int s0, int ns, int wo, const int* __restrict__ ocnt,
                                                       const int* __restrict__ eo_nb,
                                                       const double4* __restrict__ sx0,
                                                       const double4* __restrict__ su,
                                                       const double* __restrict__ L,
                                                       const double2* __restrict__ lame,
                                                       double4* __restrict__ sP, double* __restrict__ sF,
                                                       double* __restrict__ sE, double* __restrict__ sS,
                                                       int fes, int store)
{
    const int s = s0 + (int)((blockIdx.x * blockDim.x + threadIdx.x) / G);   // slots [s0, ns)
    const int g = (int)threadIdx.x & (G - 1);
    if (s >= ns) return;   // whole groups: G divides the block
    const double4 u4 = su[s];
    const double4 x0s = sx0[s];
    const double ui[3] = {u4.x, u4.y, u4.z};
    double Fr[DIM][DIM];
#pragma unroll
    for (int a = 0; a < DIM; ++a)
#pragma unroll
        for (int b = 0; b < DIM; ++b) Fr[a][b] = 0.0;
    const int cnt = ocnt[s];
    for (int k0 = g; k0 < cnt; k0 += G * U) {
        int t[U];
        double4 pr[U], uj[U], xj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = eo_nb[sell(s, wo, k0 + G * u < cnt ? k0 + G * u : cnt - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uj[u] = su[t[u]];
            xj[u] = sx0[t[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) pr[u] = struct_pair<DIM>(P, x0s, xj[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (k0 + G * u >= cnt) break;
            const double x0ij[3] = {pr[u].x, pr[u].y, pr[u].z};
            const double ujv[3] = {uj[u].x, uj[u].y, uj[u].z};
#pragma unroll
            for (int a = 0; a < DIM; ++a) {
                const double xa = x0ij[a] + (ujv[a] - ui[a]);
#pragma unroll
                for (int b = 0; b < DIM; ++b) Fr[a][b] += pr[u].w * xa * x0ij[b];
            }
        }
    }
    if (G > 1) {
#pragma unroll
        for (int a = 0; a < DIM; ++a)
#pragma unroll
            for (int b = 0; b < DIM; ++b) Fr[a][b] = group_sum<G>(Fr[a][b]);
        if (g != 0) return;
    }
    double Lm[DIM][DIM], F[DIM][DIM], E[DIM][DIM], S[DIM][DIM], PK[DIM][DIM];
#pragma unroll
    for (int a = 0; a < DIM; ++a)
#pragma unroll
        for (int b = 0; b < DIM; ++b) Lm[a][b] = L[(size_t)s * 9 + 3 * a + b];
#pragma unroll
    for (int a = 0; a < DIM; ++a)
#pragma unroll
        for (int b = 0; b < DIM; ++b) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < DIM; ++k) acc += Fr[a][k] * Lm[k][b];
            F[a][b] = acc;
        }
    double tr = 0.0;
#pragma unroll
    for (int a = 0; a < DIM; ++a)
#pragma unroll
        for (int b = 0; b < DIM; ++b) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < DIM; ++k) acc += F[k][a] * F[k][b];
            E[a][b] = 0.5 * (acc - (a == b ? 1.0 : 0.0));
            if (a == b) tr += E[a][b];
        }
    const double2 lm = lame[s];   // (lambda, mu)
#pragma unroll
    for (int a = 0; a < DIM; ++a)
#pragma unroll
        for (int b = 0; b < DIM; ++b) S[a][b] = 2.0 * lm.y * E[a][b] + (a == b ? lm.x * tr : 0.0);
    // P = F S L
#pragma unroll
    for (int a = 0; a < DIM; ++a)
#pragma unroll
        for (int b = 0; b < DIM; ++b) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < DIM; ++k)
#pragma unroll
                for (int l = 0; l < DIM; ++l) acc += F[a][k] * S[k][l] * Lm[l][b];
            PK[a][b] = acc;
        }
    if (DIM == 2) {
        sP[s] = make_double4(PK[0][0], PK[0][1], PK[1 % DIM][0], PK[1 % DIM][1 % DIM]);
    } else {
#pragma unroll
        for (int a = 0; a < DIM; ++a) sP[(size_t)s * 3 + a] = make_double4(PK[a][0], PK[a][1], PK[a][DIM - 1], 0.0);
    }
    if (!store) return;   // F, E, S are outputs only: the last substep of a batch's last step
    // element planes (StructDev): consecutive slots of the wave store one run per element; in 2-D
    // the third row and column stay the zeros set at creation
#pragma unroll
    for (int a = 0; a < DIM; ++a)
#pragma unroll
        for (int b = 0; b < DIM; ++b) {
            const size_t o = (size_t)(3 * a + b) * fes + s;
            sF[o] = F[a][b];
            sE[o] = E[a][b];
            sS[o] = S[a][b];
        }
}

// calculateStressForce (2854-2887) in gather form: v_s += dt_e/rho_s * [P_s sum_j w_sj x0_sj -
// sum_{i lists s} w_is P_i x0_is] (the reference's scatter regrouped by receiver; the first sum is
// fixed, wx0), followed by updateElasticPosition (1910-2082): module clamp, then the always-
// compiled second drift of 2070-2079 (free particles drift twice per substep; structure
// acceleration is zero).  Also refreshes the displacement u for the next substep.
// first Piola-Kirchhoff rows of slot s (2-D: one packed double4, 3-D: three rows)
template <int DIM>
__device__ __forceinline__ void struct_P(const double4* sP, int s, double (&Pm)[DIM][3])
{
    if (DIM == 2) {
        const double4 r = sP[s];
        Pm[0][0] = r.x; Pm[0][1] = r.y; Pm[0][2] = 0.0;
        Pm[1 % DIM][0] = r.z; Pm[1 % DIM][1] = r.w; Pm[1 % DIM][2] = 0.0;
    } else {
#pragma unroll
        for (int a = 0; a < DIM; ++a) {
            const double4 r = sP[(size_t)s * 3 + a];
            Pm[a][0] = r.x; Pm[a][1] = r.y; Pm[a][2] = r.z;
        }
    }
}

template <int DIM, int G, int U = MPH_US>
__global__ __launch_bounds__(256) void k_struct_velocity(DevParams P, int s0, int ns, int wi,
                                                         const int* __restrict__ icnt,
                                                         const int* __restrict__ ei_nb,
                                                         const double4* __restrict__ wx0,
                                                         const double4* __restrict__ sP,
                                                         const double* __restrict__ inv_rho,
                                                         const int* __restrict__ clamp,
                                                         const double4* __restrict__ sx0,
                                                         double4* __restrict__ sx, double4* __restrict__ sv,
                                                         double4* __restrict__ su, int last,
                                                         const int* __restrict__ bidx, Soa B,
                                                         double4* __restrict__ force)
{
    const int s = s0 + (int)((blockIdx.x * blockDim.x + threadIdx.x) / G);   // slots [s0, ns)
    const int g = (int)threadIdx.x & (G - 1);
    if (s >= ns) return;   // whole groups: G divides the block
    double dv[DIM];
#pragma unroll
    for (int a = 0; a < DIM; ++a) dv[a] = 0.0;
    if (g == 0) {   // the receiver's own half, once per slot (G > 1: added to lane 0's share)
        const double4 c = wx0[s];
        const double cv[3] = {c.x, c.y, c.z};
        double Ps[DIM][3];
        struct_P<DIM>(sP, s, Ps);
#pragma unroll
        for (int a = 0; a < DIM; ++a) {
            double f = 0.0;
#pragma unroll
            for (int b = 0; b < DIM; ++b) f += Ps[a][b] * cv[b];
            dv[a] = f;
        }
    }
    const int cnt = icnt[s];
    const double4 x0me = sx0[s];
    for (int k0 = g; k0 < cnt; k0 += G * U) {
        int t[U];
        double4 xi0[U];
        double Pi[U][DIM][3];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = ei_nb[sell(s, wi, k0 + G * u < cnt ? k0 + G * u : cnt - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            struct_P<DIM>(sP, t[u], Pi[u]);
            xi0[u] = sx0[t[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (k0 + G * u >= cnt) break;
            // the sender i's pair {x0_is, w_is} (main.cpp:2862-2880, from i's side)
            const double4 pr = struct_pair<DIM>(P, xi0[u], x0me);
            const double x0[3] = {pr.x, pr.y, pr.z};
#pragma unroll
            for (int a = 0; a < DIM; ++a) {
                double f = 0.0;
#pragma unroll
                for (int b = 0; b < DIM; ++b) f += Pi[u][a][b] * x0[b];
                dv[a] -= f * pr.w;
            }
        }
    }
    if (G > 1) {
#pragma unroll
        for (int a = 0; a < DIM; ++a) dv[a] = group_sum<G>(dv[a]);
        if (g != 0) return;
    }
    double4 v = sv[s];
    double4 xo = sx[s];
    const double ir = inv_rho[s];
    double vv[3] = {v.x, v.y, v.z};
#pragma unroll
    for (int a = 0; a < DIM; ++a) vv[a] += ir * dv[a] * P.edt;
    double xx[3] = {xo.x, xo.y, xo.z};
    const int cl = clamp[s];
    const double4 x0s = sx0[s];
    if (cl) {
        xx[0] = x0s.x; xx[1] = x0s.y; xx[2] = x0s.z;
        vv[0] = vv[1] = vv[2] = 0.0;
    } else if (P.module != MPH_MODULE_NONE) {
        for (int d = 0; d < 3; ++d) xx[d] += vv[d] * P.edt;
    }
    for (int d = 0; d < 3; ++d) xx[d] += vv[d] * P.edt;
    if (last) {
        // back into the integrated state (A order) at the entry pass B took it from
        const int r = bidx[s];
        B.x[r] = xx[0]; B.y[r] = xx[1]; B.z[r] = xx[2];
        B.vx[r] = vv[0]; B.vy[r] = vv[1]; B.vz[r] = vv[2];
        if (cl == 1) force[r] = make_double4(0.0, 0.0, 0.0, 0.0);
        return;
    }
    sv[s] = make_double4(vv[0], vv[1], vv[2], 0.0);
    const double4 xn = make_double4(xx[0], xx[1], xx[2], xo.w);
    sx[s] = xn;
    su[s] = struct_disp(P, xn, x0s);
}

// --------------------------------------------------------- elastic-solid initialisation ----
// calculateInitialNeighbor (main.cpp:1497-1658), calculateNormalizer (2544-2653) on the device.
// The structure slots (x0 in slot = file order) are binned on the GPU cell grid of the fluid
// search (cells >= rc/2, the contiguous axis halved); each slot scans the 5x5(x9) stencil of
// slot cells with the reference's exact test  q0^2+q1^2+q2^2 <= (MaxRadius+MARGIN)^2  on the
// Mod image of InitialPosition (2-D: q2 = 0, main.cpp:1605), structure j only (the binned set).
// Rows are then sorted ascending, the transpose (the senders of calculateStressForce's scatter)
// is built with atomics and sorted, and the normalizer sums run over the sorted rows in the
// host's order -- so lists, counts, Normalizer and the fixed sum w x0 equal the host build.

__global__ __launch_bounds__(256) void k_sinit_bin(DevParams P, int ns, const double4* __restrict__ x0,
                                                   int* __restrict__ key, int* __restrict__ cnt,
                                                   int* __restrict__ slot)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const double4 p = x0[s];
    const int k = cell_id(P, p.x, p.y, p.z);
    key[s] = k;
    slot[s] = atomicAdd(&cnt[k], 1);
}

// cell order, slot-ascending inside a cell (deterministic)
__global__ __launch_bounds__(256) void k_sinit_place(int ns, const int* __restrict__ key,
                                                     const int* __restrict__ slot,
                                                     const int* __restrict__ start, int* __restrict__ tmp,
                                                     int* __restrict__ sorted, int phase)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const int k = key[s];
    if (phase == 0) {
        tmp[start[k] + slot[s]] = s;
        return;
    }
    const int b = start[k], e = start[k + 1];
    int r = 0;
    for (int q = b; q < e; ++q) r += tmp[q] < s;
    sorted[b + r] = s;
}

// mode 0: count the row of every slot; mode 1: write it into the ELL tile rows (width w, stencil
// order) -- per-slot overflow (>= 512, main.cpp:1609-1611) raises the error flag
template <int DIM>
__global__ __launch_bounds__(256) void k_sinit_search(DevParams P, int ns, const double4* __restrict__ x0,
                                                      const int* __restrict__ start,
                                                      const int* __restrict__ sorted, int* __restrict__ ocnt,
                                                      int* __restrict__ ell, int w, int mode,
                                                      DevState* __restrict__ st)
{
#pragma clang fp contract(off)
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const double4 xi = x0[s];
    const int cx = cell_axis(xi.x, P.corg[0], P.dw[0], P.ginv[0], P.gc[0]);
    const int cy = cell_axis(xi.y, P.corg[1], P.dw[1], P.ginv[1], P.gc[1]);
    const int cz = DIM == 3 ? cell_axis(xi.z, P.corg[2], P.dw[2], P.ginv[2], P.gc[2]) : 0;
    // stencil half-widths in cells: kReach across (cells >= rc/kReach), P.sa along the contiguous axis
    const int ca = contig_axis(DIM, P.perm);
    const int rx = ca == 0 ? P.sa : kReach, ry = ca == 1 ? P.sa : kReach,
              rz = DIM == 3 ? (ca == 2 ? P.sa : kReach) : 0;
    int c = 0;
    for (int dx = -rx; dx <= rx; ++dx) {
        const int jx = wrap_cell(cx + dx, P.gc[0]);
        for (int dy = -ry; dy <= ry; ++dy) {
            const int jy = wrap_cell(cy + dy, P.gc[1]);
            for (int dz = -rz; dz <= rz; ++dz) {
                const int jz = DIM == 3 ? wrap_cell(cz + dz, P.gc[2]) : 0;
                const int cell = cell_index(P, jx, jy, jz);
                for (int q = start[cell], e = start[cell + 1]; q < e; ++q) {
                    const int t = sorted[q];
                    if (t == s) continue;
                    const double4 xj = x0[t];
                    const double q0 = image_exact<false>(xj.x - xi.x, P.dw[0], P.hw[0], P.w075[0]);
                    const double q1 = image_exact<false>(xj.y - xi.y, P.dw[1], P.hw[1], P.w075[1]);
                    const double q2 = DIM == 3 ? image_exact<false>(xj.z - xi.z, P.dw[2], P.hw[2], P.w075[2]) : 0.0;
                    if (r2_exact(q0, q1, q2) <= P.rc2) {
                        if (mode == 1 && c < w) ell[sell(s, w, c)] = t;
                        ++c;
                    }
                }
            }
        }
    }
    if (mode == 0) {
        ocnt[s] = c;
        if (c >= kMaxNeighbor) atomicOr(&st->overflow, 1);
    }
}

// ascending order inside each ELL row (insertion sort in place; rows are <= ~80 long)
__global__ __launch_bounds__(256) void k_sinit_sort_rows(int ns, const int* __restrict__ cnt, int* __restrict__ ell,
                                                         int w)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const int n = cnt[s];
    for (int a = 1; a < n; ++a) {
        const int v = ell[sell(s, w, a)];
        int b = a - 1;
        while (b >= 0 && ell[sell(s, w, b)] > v) {
            ell[sell(s, w, b + 1)] = ell[sell(s, w, b)];
            --b;
        }
        ell[sell(s, w, b + 1)] = v;
    }
}

// transpose: mode 0 counts the in-degree, mode 1 appends s to the in-row of every t it lists
__global__ __launch_bounds__(256) void k_sinit_transpose(int ns, const int* __restrict__ ocnt,
                                                         const int* __restrict__ eo, int wo,
                                                         int* __restrict__ icnt, int* __restrict__ ei, int wi,
                                                         int mode)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const int n = ocnt[s];
    for (int k = 0; k < n; ++k) {
        const int t = eo[sell(s, wo, k)];
        const int pos = atomicAdd(&icnt[t], 1);
        if (mode == 1) ei[sell(t, wi, pos)] = s;
    }
}

// calculateNormalizer (main.cpp:2555-2651) over the sorted row: the 3x3 accumulation in both
// dimensions (the TWO_DIMENSION typo of 2545), 2-D inverse with the identity fallback, 3-D
// cofactor inverse (left unchanged when det = 0, like the reference); plus the fixed sum of
// w_sj x0_sj that the P_s half of the gather-form stress force uses
template <int DIM>
__global__ __launch_bounds__(256) void k_sinit_normalizer(DevParams P, int ns, const double4* __restrict__ x0,
                                                          const int* __restrict__ ocnt,
                                                          const int* __restrict__ eo, int wo,
                                                          double* __restrict__ L, double4* __restrict__ wx0)
{
#pragma clang fp contract(off)
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const double4 xi = x0[s];
    double N[3][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
    double c3[3] = {0.0, 0.0, 0.0};
    const int n = ocnt[s];
    for (int k = 0; k < n; ++k) {
        const double4 xj = x0[eo[sell(s, wo, k)]];
        const double4 pr = struct_pair<DIM>(P, xi, xj);
        // the accumulation runs over all three components: in 2-D the z image of equal z is 0
        const double q[3] = {pr.x, pr.y, image_exact<false>(xj.z - xi.z, P.dw[2], P.hw[2], P.w075[2])};
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) N[a][b] += pr.w * q[a] * q[b];
        c3[0] += pr.w * pr.x;
        c3[1] += pr.w * pr.y;
        c3[2] += pr.w * pr.z;
    }
    if (DIM == 2) {
        const double a = N[0][0], b = N[0][1], cc = N[1][0], d = N[1][1];
        const double det = a * d - b * cc;
        if (det != 0.0) {
            N[0][0] = d / det; N[0][1] = -b / det; N[1][0] = -cc / det; N[1][1] = a / det;
        } else {
            N[0][0] = 1.0; N[0][1] = 0.0; N[1][0] = 0.0; N[1][1] = 1.0;
        }
    } else {
        const double det = N[0][0] * (N[1][1] * N[2][2] - N[1][2] * N[2][1])
                         - N[0][1] * (N[1][0] * N[2][2] - N[1][2] * N[2][0])
                         + N[0][2] * (N[1][0] * N[2][1] - N[1][1] * N[2][0]);
        if (det != 0.0) {
            double adj[3][3];
            adj[0][0] = N[1][1] * N[2][2] - N[1][2] * N[2][1];
            adj[0][1] = -N[1][0] * N[2][2] + N[1][2] * N[2][0];
            adj[0][2] = N[1][0] * N[2][1] - N[1][1] * N[2][0];
            adj[1][0] = -N[0][1] * N[2][2] + N[0][2] * N[2][1];
            adj[1][1] = N[0][0] * N[2][2] - N[0][2] * N[2][0];
            adj[1][2] = -N[0][0] * N[2][1] + N[0][1] * N[2][0];
            adj[2][0] = N[0][1] * N[1][2] - N[0][2] * N[1][1];
            adj[2][1] = -N[0][0] * N[1][2] + N[0][2] * N[1][0];
            adj[2][2] = N[0][0] * N[1][1] - N[0][1] * N[1][0];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) N[a][b] = adj[a][b] / det;
        }
    }
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) L[(size_t)s * 9 + 3 * a + b] = N[a][b];
    wx0[s] = make_double4(c3[0], c3[1], c3[2], 0.0);
}

// ------------------------------------------------------------------ slab decomposition -----
// Multi-GPU redistribution (mph_dist.hip).  Every B entry is classified by its slab coordinate
// after this step's wall motion + periodic wrap; a stable partition then writes the owned and
// outgoing particles into C as [migrate R | band R | inner | band L | migrate L] (ghosts of the
// previous step are dropped).  Migrants keep a copy here as ghosts (id -> -1-id).

__device__ __forceinline__ unsigned long long lanemask_lt() { return (1ull << (threadIdx.x & 63)) - 1ull; }

__device__ __forceinline__ bool dist_sends(int c) { return c == kMigR || c == kBandR || c == kBandL || c == kMigL; }
constexpr int kMsgHeader = 16;   // redistribution message header: the two class counts

// wface (early send, see k_dist_early_classify): the face wavefronts of the previous step, whose
// particles were moved and sent already -- not moved again here, and no other particle may be
// of a sending class (it would have moved more than the face margin: an error)
__global__ __launch_bounds__(256) void k_dist_classify(DevParams P, DevState* __restrict__ st, SlabGeom g,
                                                       Soa B, const DistLayout* __restrict__ lay, int move,
                                                       int* __restrict__ cls, int* __restrict__ bcnt, int nb,
                                                       const int* __restrict__ wface)
{
    __shared__ int wc[4][kSlabClasses];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = lay->n;   // entries of B: the previous redistribution's count
    int c = -1;
    if (p < n) {
        if (B.id[p] < 0) {
            c = kSlabDrop;
        } else {
            const bool face = wface && wface[p >> 6] == 1;
            double x = B.x[p], y = B.y[p], z = B.z[p];
            if (move && !face) move_and_wrap(P, st, B, p, x, y, z);
            const double a = g.axis == 0 ? x : (g.axis == 1 ? y : z);
            c = dev_is_struct(B.type[p]) ? slab_class_static(g, a) : slab_class(g, a);
            if (c == kSlabLost) {
                atomicOr(&st->overflow, 2);
                c = kInner;
            }
            if (wface && !face && dist_sends(c)) atomicOr(&st->overflow, 8);
        }
        cls[p] = c;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kSlabClasses; ++k) {
        const unsigned long long m = __ballot(c == k);
        if (lane == 0) wc[wave][k] = __popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < kSlabClasses) {
        int t = 0;
        for (int w = 0; w < 4; ++w) t += wc[w][threadIdx.x];
        bcnt[threadIdx.x * nb + blockIdx.x] = t;
    }
}

// Early send (mph_dist.hip): at the end of a step, once pass B has integrated the face wavefronts
// (wface, written by pass B), their owned particles are moved (calculateWall / periodic wrap, as
// k_dist_classify would at the next step) and classified; the others count as nothing here.
__global__ __launch_bounds__(256) void k_dist_early_classify(DevParams P, DevState* __restrict__ st, SlabGeom g,
                                                             Soa B, const DistLayout* __restrict__ lay,
                                                             const int* __restrict__ wface,
                                                             int* __restrict__ cls, int* __restrict__ bcnt, int nb)
{
    __shared__ int wc[4][kSlabClasses];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = lay->n;
    int c = -1;
    if (p < n && B.id[p] >= 0 && wface[p >> 6] == 1) {
        double x = B.x[p], y = B.y[p], z = B.z[p];
        move_and_wrap(P, st, B, p, x, y, z);
        const double a = g.axis == 0 ? x : (g.axis == 1 ? y : z);
        c = dev_is_struct(B.type[p]) ? slab_class_static(g, a) : slab_class(g, a);   // as k_dist_classify
        if (c == kSlabLost) c = kInner;   // reported by k_dist_classify at the next step
    }
    if (p < n) cls[p] = c;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kSlabClasses; ++k) {
        const unsigned long long m = __ballot(c == k);
        if (lane == 0) wc[wave][k] = __popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < kSlabClasses) {
        int t = 0;
        for (int w = 0; w < 4; ++w) t += wc[w][threadIdx.x];
        bcnt[threadIdx.x * nb + blockIdx.x] = t;
    }
}

// The messages straight from B, in the order k_dist_scatter + k_dist_pack give them (stable by
// B index within each class): to the left [bandL | migL], to the right [migR | bandR], each behind
// its count header; migrants travel with negated ids, as from C.
__global__ __launch_bounds__(256) void k_dist_early_pack(Soa B, DistLayout* __restrict__ lay,
                                                         const int* __restrict__ cls,
                                                         const int* __restrict__ boff, int nb, int cap_l,
                                                         int cap_r, DevState* __restrict__ st,
                                                         char* __restrict__ buf_l, char* __restrict__ buf_r)
{
    __shared__ int wc[4][kSlabClasses];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = lay->n;
    const int c = p < n ? cls[p] : -1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int rank = 0;
#pragma unroll
    for (int k = 0; k < kSlabClasses; ++k) {
        const unsigned long long m = __ballot(c == k);
        if (c == k) rank = __popcll(m & lanemask_lt());
        if (lane == 0) wc[wave][k] = __popcll(m);
    }
    __syncthreads();
    const int sMigR = boff[kMigR * nb], sBandR = boff[kBandR * nb], sInner = boff[kInner * nb];
    const int sBandL = boff[kBandL * nb], sMigL = boff[kMigL * nb], sDrop = boff[kSlabDrop * nb];
    const int mr = sInner - sMigR, ml = sDrop - sBandL;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int* hl = (int*)buf_l;
        int* hr = (int*)buf_r;
        hl[0] = sMigL - sBandL; hl[1] = sDrop - sMigL;   // {bandL, migL}
        hr[0] = sBandR - sMigR; hr[1] = sInner - sBandR; // {migR, bandR}
        lay->send[0] = hl[0]; lay->send[1] = hl[1]; lay->send[2] = hr[0]; lay->send[3] = hr[1];
        atomicMax(&lay->hw[0], min(ml, cap_l));
        atomicMax(&lay->hw[1], min(mr, cap_r));
        if (ml > cap_l || mr > cap_r) atomicOr(&st->overflow, 8);
    }
    if (!dist_sends(c)) return;
    int o = boff[c * nb + blockIdx.x] + rank;
    for (int w = 0; w < wave; ++w) o += wc[w][c];
    const bool left = c == kBandL || c == kMigL;
    // the stride is clamped to the capacity like k_dist_pack's (the header keeps the true counts,
    // so a receiver skips an overfull message): an overflow is MPH_ERR_CAPACITY, never a write
    // past the buffer
    const int cap = left ? cap_l : cap_r;
    const int m = min(left ? ml : mr, cap);
    const int j = left ? o - sBandL : o - sMigR;
    if (j >= m) return;
    double* d = (double*)((left ? buf_l : buf_r) + kMsgHeader);
    int* q = (int*)(d + 6 * (size_t)m);
    d[j] = B.x[p]; d[m + j] = B.y[p]; d[2 * m + j] = B.z[p];
    d[3 * m + j] = B.vx[p]; d[4 * m + j] = B.vy[p]; d[5 * m + j] = B.vz[p];
    q[j] = B.type[p];
    const int id = B.id[p];
    q[m + j] = (c == kMigR || c == kMigL) ? -1 - id : id;
}

// also writes the layout's send counts (left-going {bandL, migL}, right-going {migR, bandR}) from
// the class starts (block 0), which the pack kernels and the count exchange of mph_create read
__global__ __launch_bounds__(256) void k_dist_scatter(Soa B, DistLayout* __restrict__ lay,
                                                      const int* __restrict__ cls,
                                                      const int* __restrict__ boff, int nb, Soa C,
                                                      int* __restrict__ dseg, int* __restrict__ vidx)
{
    __shared__ int wc[4][kSlabClasses];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = lay->n;
    const int c = p < n ? cls[p] : -1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int rank = 0;
#pragma unroll
    for (int k = 0; k < kSlabClasses; ++k) {
        const unsigned long long m = __ballot(c == k);
        if (c == k) rank = __popcll(m & lanemask_lt());
        if (lane == 0) wc[wave][k] = __popcll(m);
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x <= kSlabClasses) dseg[threadIdx.x] = boff[threadIdx.x * nb];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        auto len = [&](int k) { return boff[(k + 1) * nb] - boff[k * nb]; };
        lay->send[0] = len(kBandL);
        lay->send[1] = len(kMigL);
        lay->send[2] = len(kMigR);
        lay->send[3] = len(kBandR);
    }
    if (c < 0 || c == kSlabDrop) return;
    int o = boff[c * nb + blockIdx.x] + rank;
    for (int w = 0; w < wave; ++w) o += wc[w][c];
    if (vidx) {   // VSrc: only where the entry lives
        vidx[o] = (c == kMigR || c == kMigL) ? -1 - p : p;
        return;
    }
    C.x[o] = B.x[p]; C.y[o] = B.y[p]; C.z[o] = B.z[p];
    C.vx[o] = B.vx[p]; C.vy[o] = B.vy[p]; C.vz[o] = B.vz[p];
    C.type[o] = B.type[p];
    const int id = B.id[p];
    C.id[o] = (c == kMigR || c == kMigL) ? -1 - id : id;
}

// Messages of a redistribution travel with a fixed capacity (so the exchange has host-known
// sizes and can sit inside a captured graph); the live counts are the 2-int count messages.
// side 0: [bandL | migL] to the left, side 1: [migR | bandR] to the right.
__device__ __forceinline__ void dist_send_range(const DistLayout* lay, int side, int& off, int& m)
{
    off = side == 0 ? lay->seg[kBandL] : lay->seg[kMigR];
    m = side == 0 ? lay->send[0] + lay->send[1] : lay->send[2] + lay->send[3];
}

// side 0: from the left (their {migR, bandR}) appended at nc, side 1: from the right after it;
// r[4] = the received counts (the message headers)
__device__ __forceinline__ void dist_recv_range(const DistLayout* lay, const int* r, int side, int& off, int& m)
{
    const int nc = lay->seg[kSlabDrop];
    const int fl = r[0] + r[1];
    off = side == 0 ? nc : nc + fl;
    m = side == 0 ? fl : r[2] + r[3];
}

// message layout: a 16-byte header with the two class counts (so no separate count message is
// needed per step), then x[m] y[m] z[m] vx[m] vy[m] vz[m] (double) type[m] id[m] (int), 56 B per
// particle (kMsgHeader above)
// both messages in one launch: blockIdx.y = side
__global__ __launch_bounds__(256) void k_dist_pack(Soa C, DistLayout* __restrict__ lay, int cap_l, int cap_r,
                                                   DevState* __restrict__ st, char* __restrict__ buf_l,
                                                   char* __restrict__ buf_r, VSrc vs)
{
    const int side = blockIdx.y;
    const int cap = side ? cap_r : cap_l;
    char* buf = side ? buf_r : buf_l;
    int off, m;
    dist_send_range(lay, side, off, m);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int* h = (int*)buf;
        h[0] = lay->send[2 * side];
        h[1] = lay->send[2 * side + 1];
    }
    if (m > cap) {   // more than the message capacity: an error (MPH_ERR_CAPACITY), never a fault
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&st->overflow, 8);
        m = cap;
    }
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicMax(&lay->hw[side], m);
    if (k >= m) return;
    double* d = (double*)(buf + kMsgHeader);
    int* q = (int*)(d + 6 * (size_t)m);
    Soa S;
    bool mig;
    const int s = vsrc_entry(vs, C, off + k, S, mig);   // the sent classes are all kept entries
    d[k] = S.x[s]; d[m + k] = S.y[s]; d[2 * m + k] = S.z[s];
    d[3 * m + k] = S.vx[s]; d[4 * m + k] = S.vy[s]; d[5 * m + k] = S.vz[s];
    q[k] = S.type[s];
    q[m + k] = mig ? -1 - S.id[s] : S.id[s];
}

// received message -> C[off, off+m); ownership flips (their migrants are ours, their band
// particles are our ghosts): id -> -1-id for every entry.  The right-hand message completes the
// layout: n = kept + received, n_own = the kept owned classes + the received migrants.
// both messages in one launch: blockIdx.y = side (0 from the left with capacity cap_l, 1 from the right)
__global__ __launch_bounds__(256) void k_dist_unpack(const char* __restrict__ buf_l, const char* __restrict__ buf_r,
                                                     DistLayout* __restrict__ lay, int cap_l, int cap_r, int cap,
                                                     DevState* __restrict__ st, Soa C)
{
    const int side = blockIdx.y;
    const int cap_msg = side ? cap_r : cap_l;
    // the received counts, from the two message headers (from the left: {migR, bandR} of the left
    // neighbour, from the right: {bandL, migL} of the right neighbour)
    const int* hl = (const int*)buf_l;
    const int* hr = (const int*)buf_r;
    const int r[4] = {hl[0], hl[1], hr[0], hr[1]};
    const char* buf = side == 0 ? buf_l : buf_r;
    int off, m;
    dist_recv_range(lay, r, side, off, m);
    const int mm = m;   // the sender's count = the stride of its message
    const bool first = blockIdx.x == 0 && threadIdx.x == 0;
    if (mm > cap_msg || off + m > cap) {   // the sender flagged it too; read nothing out of range
        if (first) atomicOr(&st->overflow, 8);
        m = mm > cap_msg ? 0 : max(0, min(m, cap - off));
    }
    if (first) {
        atomicMax(&lay->hw[2 + side], mm);
        if (side == 0) {
            // the layout's receive counts, for the halo ranges of this step
            lay->recv[0] = r[0]; lay->recv[1] = r[1]; lay->recv[2] = r[2]; lay->recv[3] = r[3];
        } else {
            const int* seg = lay->seg;
            const int n = min(off + m, cap);
            lay->n = n;
            lay->n_own = (seg[kBandR + 1] - seg[kBandR]) + (seg[kInner + 1] - seg[kInner]) +
                         (seg[kBandL + 1] - seg[kBandL]) + r[0] + r[3];
            atomicMax(&lay->hw[4], off + (r[2] + r[3]));
        }
    }
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const double* d = (const double*)(buf + kMsgHeader);
    const int* q = (const int*)(d + 6 * (size_t)mm);
    const int s = off + k;
    C.x[s] = d[k]; C.y[s] = d[mm + k]; C.z[s] = d[2 * mm + k];
    C.vx[s] = d[3 * mm + k]; C.vy[s] = d[4 * mm + k]; C.vz[s] = d[5 * mm + k];
    C.type[s] = q[k];
    C.id[s] = -1 - q[mm + k];
}

// Elastic ghost slots (slab mode): w double4 rows per slot, slot k of the message = idx[k].
__global__ __launch_bounds__(256) void k_struct_pack(const double4* __restrict__ src, int w,
                                                     const int* __restrict__ idx, int m,
                                                     double4* __restrict__ buf)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m * w) return;
    const int k = t / w, r = t - k * w;
    buf[t] = src[(size_t)idx[k] * w + r];
}

__global__ __launch_bounds__(256) void k_struct_unpack(const double4* __restrict__ buf, int w,
                                                       const int* __restrict__ idx, int m,
                                                       double4* __restrict__ dst)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m * w) return;
    const int k = t / w, r = t - k * w;
    dst[(size_t)idx[k] * w + r] = buf[t];
}

// C-index ranges of the pass-A halo (mph_dist.hip step 5), from the device layout: dir 0 = to the
// left [the left neighbour's migrants we now own | our band-left], 1 = to the right [the right
// neighbour's migrants we now own | our band-right], 2 = from the left [our migrants that went
// left | the left neighbour's band-right ghosts], 3 = from the right (mirror image).
__device__ __forceinline__ void halo_ranges(const DistLayout* L, int dir, int& o1, int& n1, int& o2, int& n2)
{
    const int* seg = L->seg;
    const int nc = seg[kSlabDrop];
    const int fl = L->recv[0] + L->recv[1];
    if (dir == 0) { o1 = nc; n1 = L->recv[0]; o2 = seg[kBandL]; n2 = seg[kBandL + 1] - seg[kBandL]; }
    else if (dir == 1) { o1 = nc + fl + L->recv[2]; n1 = L->recv[3]; o2 = seg[kBandR]; n2 = seg[kBandR + 1] - seg[kBandR]; }
    else if (dir == 2) { o1 = seg[kMigL]; n1 = seg[kMigL + 1] - seg[kMigL]; o2 = nc + L->recv[0]; n2 = L->recv[1]; }
    else { o1 = seg[kMigR]; n1 = seg[kMigR + 1] - seg[kMigR]; o2 = nc + fl; n2 = L->recv[2]; }
}

// pass-A values of two C-index ranges, read at their sorted position dst_of[c]; cap bounds the
// message (the counts are within it once the redistribution's capacity checks passed)
// both directions in one launch: dir = blockIdx.y (0 to the left into buf_a with capacity cap_a,
// 1 to the right into buf_b)
__global__ __launch_bounds__(256) void k_halo_pack(const int* __restrict__ dst_of, const DistLayout* __restrict__ lay,
                                                   int cap_a, int cap_b, HaloFields F, double* __restrict__ buf_a,
                                                   double* __restrict__ buf_b)
{
    const int dir = blockIdx.y;
    const int cap = dir ? cap_b : cap_a;
    double* buf = dir ? buf_b : buf_a;
    int o1, n1, o2, n2;
    halo_ranges(lay, dir, o1, n1, o2, n2);
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = min(n1 + n2, cap);
    if (k >= m) return;
    const int a = dst_of[k < n1 ? o1 + k : o2 + (k - n1)];
    for (int f = 0; f < F.nf; ++f) buf[(size_t)f * m + k] = F.f[f][a];
}

// both directions in one launch: dir = 2 + blockIdx.y (2 from the left out of buf_a, 3 from the right)
__global__ __launch_bounds__(256) void k_halo_unpack(const double* __restrict__ buf_a, const double* __restrict__ buf_b,
                                                     const int* __restrict__ dst_of, const DistLayout* __restrict__ lay,
                                                     int cap_a, int cap_b, HaloFields F)
{
    const int dir = 2 + blockIdx.y;
    const int cap = blockIdx.y ? cap_b : cap_a;
    const double* buf = blockIdx.y ? buf_b : buf_a;
    int o1, n1, o2, n2;
    halo_ranges(lay, dir, o1, n1, o2, n2);
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int m = min(n1 + n2, cap);
    if (k >= m) return;
    const int a = dst_of[k < n1 ? o1 + k : o2 + (k - n1)];
    for (int f = 0; f < F.nf; ++f) F.f[f][a] = buf[(size_t)f * m + k];
    if (F.rec) rec_store_p(F.rec, F.rec_stride, a, buf[k]);
}

// ---------------------------------------------------------------------------- launchers -----

static inline int blocks(int n, int t) { return (n + t - 1) / t; }

// Grid of the two list passes: the XCD map (list_block) needs a multiple of 8 blocks, with 25 %
// slack for its unequal ranges.  Below Launch.xcd_bal_min particles (default 2^20) the split
// kernel's ~7 us costs more than the balance gains (Bar 400k, 0.23 ms per step: 1.76e9 p-steps/s
// with it, 1.80e9 without), so the passes keep the equal ranges and the search feeds no histogram.
static inline int list_grid(int n)
{
    const int nb = blocks(n, MPH_LB);
    return (nb + nb / 4 + 15) / 8 * 8;
}

// A profiled launch (mph_profile_steps): its start/stop events come from the kernel's dispatch
// packet (hipExtLaunchKernelGGL), or are recorded around it (Profiler::events).  Direct launches
// run ~9 us apart and start with a written-back L2, so they take 3-8 % longer than the same
// kernels replayed from a graph (profiles/r05/final/prof: rocprofv3 trace); mph_profile_graphs
// times the list kernels as graph replays.
#define MPH_LAUNCH(name, stream, kernel, grid, block, shm, strm, ...)                          \
    do {                                                                                       \
        if (prof) {                                                                            \
            hipEvent_t _a, _b;                                                                 \
            if (prof->events(name, stream, &_a, &_b)) {                                        \
                hipExtLaunchKernelGGL(kernel, grid, block, shm, strm, _a, _b, 0u, __VA_ARGS__); \
            } else {                                                                           \
                (void)hipEventRecord(_a, strm);                                                \
                hipLaunchKernelGGL(kernel, grid, block, shm, strm, __VA_ARGS__);               \
                (void)hipEventRecord(_b, strm);                                                \
            }                                                                                  \
        } else {                                                                               \
            hipLaunchKernelGGL(kernel, grid, block, shm, strm, __VA_ARGS__);                   \
        }                                                                                      \
    } while (0)

void launch_sort(const Launch& L, int mode)
{
    Profiler* prof = L.prof;
    const DevParams& P = *L.P;
    const int n = P.n;
    if (n == 0) return;
    const int nb = blocks(P.ncell, kScanBlock);
    const int top = nb <= kScanFusedTop;
    const int split = n >= L.xcd_bal_min;   // the passes' XCD split (list_grid, k_rank_scatter)
    MPH_LAUNCH("prep", L.stream, k_prep, dim3(blocks(n, 256)), dim3(256), 0, L.stream, P, L.st, L.B, L.key,
               L.slot, L.cnt, mode, L.vsrc);
    MPH_LAUNCH("scan_reduce", L.stream, k_scan_reduce, dim3(nb), dim3(kScanThreads), 0, L.stream, L.cnt, P.ncell,
               L.bsum);
    if (!top) MPH_LAUNCH("scan_top", L.stream, k_scan_top, dim3(1), dim3(1024), 0, L.stream, L.bsum, nb);
    MPH_LAUNCH("scan_down", L.stream, k_scan_down, dim3(nb), dim3(kScanThreads), 0, L.stream, L.cnt, P.ncell,
               L.bsum, L.start, n, P.n_dev, top);
    MPH_LAUNCH("place", L.stream, k_place, dim3(blocks(n, 256)), dim3(256), 0, L.stream, P, L.st, L.key,
               L.slot, L.start, L.tmp, mode);
    MPH_LAUNCH("rank_scatter", L.stream, k_rank_scatter, dim3(blocks(n, 256)), dim3(256), 0, L.stream, P,
               L.key, L.start, L.tmp, L.B, L.A, L.rank_of, L.dst_of, mode, L.vsrc, L.st, split);
}

static PassAOut pass_a_out(const Launch& L)
{
    return PassAOut{L.pres, L.gx, L.gy, L.gz, L.pa, L.dens_a, L.vstrain, L.divp, L.fpart, L.rec};
}

void launch_neighbors(const Launch& L)
{
    Profiler* prof = L.prof;
    const DevParams& P = *L.P;
    if (P.n == 0) return;
    const int bal = P.n >= L.xcd_bal_min;
#define MPH_NEIGHBORS(D, PERM)                                                                             \
    MPH_LAUNCH("neighbors", L.stream, (k_neighbors<D, PERM>), dim3(blocks(P.n, MPH_LB)), dim3(MPH_LB), 0, \
               L.stream, P, L.A, L.start, L.nbr, L.ncount, L.nbcount, L.lhdr, L.lgap, L.st, L.wface, bal)
    if (P.dim == 3) {
        switch (P.perm) {
        case 1: MPH_NEIGHBORS(3, 1); break;
        case 2: MPH_NEIGHBORS(3, 2); break;
        case 3: MPH_NEIGHBORS(3, 3); break;
        case 4: MPH_NEIGHBORS(3, 4); break;
        default: MPH_NEIGHBORS(3, 0); break;
        }
    } else {
        MPH_NEIGHBORS(2, 0);
    }
#undef MPH_NEIGHBORS
}

void launch_pass_a(const Launch& L)
{
    Profiler* prof = L.prof;
    const DevParams& P = *L.P;
    if (P.n == 0) return;
    const PassAOut po = pass_a_out(L);
    if (P.dim == 3)
        MPH_LAUNCH("pass_a", L.stream, k_pass_a<3>, dim3(list_grid(P.n)), dim3(MPH_LB), 0, L.stream, P, L.T, L.A,
                   L.nbr, L.ncount, L.lhdr, L.lgap, po, L.st);
    else
        MPH_LAUNCH("pass_a", L.stream, k_pass_a<2>, dim3(list_grid(P.n)), dim3(MPH_LB), 0, L.stream, P, L.T, L.A,
                   L.nbr, L.ncount, L.lhdr, L.lgap, po, L.st);
}

// calculateNeighbor + the pass-A sums
void launch_search_pass_a(const Launch& L)
{
    launch_neighbors(L);
    launch_pass_a(L);
}

static StructHook struct_hook(const Launch& L)
{
    StructHook h{};
    if (L.P->n_struct > 0 && L.S && L.S->slot_of) {
        h.slot_of = L.S->slot_of;
        h.sx = L.S->x;
        h.sv = L.S->v;
        h.su = L.S->u;
        h.sx0 = L.S->x0;
        h.bidx = L.S->bidx;
    }
    return h;
}

void launch_pass_b(const Launch& L, int phase)
{
    Profiler* prof = L.prof;
    const DevParams& P = *L.P;
    if (P.n == 0) return;
    // pass B reads GravityCenter and PressureA of every neighbour with surface tension; enqueue_step
    // may leave them unstored on the non-last steps of a batch only without it
    if (P.surface && !(L.gx && L.gy && L.gz && L.pa)) {
        std::fprintf(stderr, "mph: launch_pass_b with surface tension needs GravityCenter/PressureA\n");
        std::abort();
    }
#define MPH_PASS_B(S, D)                                                                            \
    MPH_LAUNCH(phase == 2 ? "pass_b_face" : "pass_b", L.stream, (k_pass_b<S, D>), dim3(list_grid(P.n)), dim3(MPH_LB), 0, L.stream, P, \
               L.T, L.A, L.rec, L.fpart, L.gx, L.gy, L.gz, L.pa, L.nbr, L.ncount, L.lhdr, L.lgap, L.force, L.acc, L.B, \
               phase, L.wface, \
               struct_hook(L), L.st)
    if (P.surface) {
        if (P.dim == 3) MPH_PASS_B(true, 3); else MPH_PASS_B(true, 2);
    } else {
        if (P.dim == 3) MPH_PASS_B(false, 3); else MPH_PASS_B(false, 2);
    }
#undef MPH_PASS_B
}

void launch_virial(const Launch& L, const Soa& X, double* vir, double* vpres)
{
    Profiler* prof = L.prof;
    const DevParams& P = *L.P;
    if (P.n == 0) return;
    if (P.dim == 3)
        MPH_LAUNCH("virial", L.stream, k_virial<3>, dim3(blocks(P.n, 256)), dim3(256), 0, L.stream, P, L.T, L.A, X,
                   L.pres, L.pa, L.gx, L.gy, L.gz, L.nbr, L.ncount, L.lhdr, L.lgap, vir, vpres);
    else
        MPH_LAUNCH("virial", L.stream, k_virial<2>, dim3(blocks(P.n, 256)), dim3(256), 0, L.stream, P, L.T, L.A, X,
                   L.pres, L.pa, L.gx, L.gy, L.gz, L.nbr, L.ncount, L.lhdr, L.lgap, vir, vpres);
}

// lanes per structure slot: one lane per slot while the launch has >= kStructLanesTarget lanes
// (eight waves per SIMD), else the smallest power of two up to 4 that reaches it -- a few ten
// thousand slots (a gate, a rank's share of one) would otherwise run one long serial list loop per
// lane on a fraction of the SIMDs.  Same box (profiles/r03/struct_lanes/): FSI gate (40 k slots,
// 3-D) stress + velocity 0.089 ms at 1 lane, 0.052 at 4, 0.055 at 8; Bar (400 k slots, 2-D)
// 0.094 at 1, 0.091 at 2, 0.102 at 4.  MPH_STRUCT_LANES=1|2|4|8 fixes it (A/B timing, tests).
constexpr long kStructLanesTarget = 8L * 1024 * 64;

int struct_lanes(int nslots)
{
    const char* e = std::getenv("MPH_STRUCT_LANES");   // read per launch (graphs capture once)
    const int forced = e ? std::atoi(e) : 0;
    if (forced == 1 || forced == 2 || forced == 4 || forced == 8) return forced;
    int g = 1;
    while (g < 4 && (long)nslots * g < kStructLanesTarget) g *= 2;
    return g;
}

#define MPH_STRUCT_G(G, D, KERNEL, NAME, ...)                                                     \
    MPH_LAUNCH(NAME, L.stream, (KERNEL<D, G>), dim3(blocks((s1 - s0) * G, 256)), dim3(256), 0,   \
               L.stream, __VA_ARGS__)
#define MPH_STRUCT_DISPATCH(KERNEL, NAME, ...)                                                    \
    do {                                                                                          \
        const int lanes = struct_lanes(S.n_own);   /* not the range: the halves sum alike */     \
        if (P.dim == 3) {                                                                         \
            switch (lanes) {                                                                      \
            case 8: MPH_STRUCT_G(8, 3, KERNEL, NAME, __VA_ARGS__); break;                         \
            case 4: MPH_STRUCT_G(4, 3, KERNEL, NAME, __VA_ARGS__); break;                         \
            case 2: MPH_STRUCT_G(2, 3, KERNEL, NAME, __VA_ARGS__); break;                         \
            default: MPH_STRUCT_G(1, 3, KERNEL, NAME, __VA_ARGS__); break;                        \
            }                                                                                     \
        } else {                                                                                  \
            switch (lanes) {                                                                      \
            case 8: MPH_STRUCT_G(8, 2, KERNEL, NAME, __VA_ARGS__); break;                         \
            case 4: MPH_STRUCT_G(4, 2, KERNEL, NAME, __VA_ARGS__); break;                         \
            case 2: MPH_STRUCT_G(2, 2, KERNEL, NAME, __VA_ARGS__); break;                         \
            default: MPH_STRUCT_G(1, 2, KERNEL, NAME, __VA_ARGS__); break;                        \
            }                                                                                     \
        }                                                                                         \
    } while (0)

void launch_struct_stress(const Launch& L, bool store, int s0, int s1)
{
    Profiler* prof = L.prof;
    const DevParams& P = *L.P;
    const StructDev& S = *L.S;
    if (s1 < 0) s1 = S.n_own;
    if (s1 <= s0) return;
    MPH_STRUCT_DISPATCH(k_struct_stress, "struct_stress", P, s0, s1, S.wo, S.ocnt, S.eo_nb, S.x0, S.u, S.L,
                        S.lame, S.P, S.F, S.E, S.S, S.fes, store ? 1 : 0);
}

void launch_struct_velocity(const Launch& L, bool last, int s0, int s1)
{
    Profiler* prof = L.prof;
    const DevParams& P = *L.P;
    const StructDev& S = *L.S;
    if (s1 < 0) s1 = S.n_own;
    if (s1 <= s0) return;
    MPH_STRUCT_DISPATCH(k_struct_velocity, "struct_velocity", P, s0, s1, S.wi, S.icnt, S.ei_nb, S.wx0, S.P,
                        S.inv_rho, S.clamp, S.x0, S.x, S.v, S.u, last ? 1 : 0, S.bidx, L.B, L.force);
}
#undef MPH_STRUCT_DISPATCH
#undef MPH_STRUCT_G

void launch_structure(const Launch& L, bool last)
{
    if (L.P->n_struct == 0) return;
    for (int sub = 0; sub < L.P->substeps; ++sub) {
        const bool final_sub = sub == L.P->substeps - 1;
        launch_struct_stress(L, last && final_sub);
        launch_struct_velocity(L, final_sub);
    }
}

int launch_struct_init(const Launch& L, int ns, const double4* x0, int* key, int* slot, int* tmp, int* sorted,
                       int* ocnt, int* icnt, int** eo, int* wo, int** ei, int* wi, double* Lm, double4* wx0,
                       void* (*alloc)(void*, size_t), void* actx)
{
    Profiler* prof = L.prof;
    const DevParams& P = *L.P;
    if (ns <= 0) return 0;
    const dim3 g(blocks(ns, 256)), b(256);
    // bin the slots on the grid (L.cnt is zero between steps and the scan re-zeroes it)
    MPH_LAUNCH("sinit_bin", L.stream, k_sinit_bin, g, b, 0, L.stream, P, ns, x0, key, L.cnt, slot);
    launch_scan(L.cnt, P.ncell, L.bsum, L.start, ns, L.stream, prof);
    MPH_LAUNCH("sinit_place", L.stream, k_sinit_place, g, b, 0, L.stream, ns, key, slot, L.start, tmp, sorted, 0);
    MPH_LAUNCH("sinit_place", L.stream, k_sinit_place, g, b, 0, L.stream, ns, key, slot, L.start, tmp, sorted, 1);
    if (P.dim == 3)
        MPH_LAUNCH("sinit_search", L.stream, k_sinit_search<3>, g, b, 0, L.stream, P, ns, x0, L.start, sorted, ocnt,
                   (int*)nullptr, 0, 0, L.st);
    else
        MPH_LAUNCH("sinit_search", L.stream, k_sinit_search<2>, g, b, 0, L.stream, P, ns, x0, L.start, sorted, ocnt,
                   (int*)nullptr, 0, 0, L.st);
    // ELL width = the longest row (one host read at initialisation)
    std::vector<int> h(ns);
    if (hipMemcpyAsync(h.data(), ocnt, sizeof(int) * ns, hipMemcpyDeviceToHost, L.stream) != hipSuccess ||
        hipStreamSynchronize(L.stream) != hipSuccess)
        return -1;
    int w = 1;
    for (int v : h) w = v > w ? v : w;
    if (w >= kMaxNeighbor) return -2;
    const size_t ntile = ((size_t)ns + 63) / 64;
    *eo = (int*)alloc(actx, ntile * w * 64 * sizeof(int));
    if (!*eo) return -3;
    if (hipMemsetAsync(*eo, 0, ntile * w * 64 * sizeof(int), L.stream) != hipSuccess) return -1;
    if (P.dim == 3)
        MPH_LAUNCH("sinit_search", L.stream, k_sinit_search<3>, g, b, 0, L.stream, P, ns, x0, L.start, sorted, ocnt,
                   *eo, w, 1, L.st);
    else
        MPH_LAUNCH("sinit_search", L.stream, k_sinit_search<2>, g, b, 0, L.stream, P, ns, x0, L.start, sorted, ocnt,
                   *eo, w, 1, L.st);
    MPH_LAUNCH("sinit_sort_rows", L.stream, k_sinit_sort_rows, g, b, 0, L.stream, ns, ocnt, *eo, w);
    *wo = w;
    // transpose: in-degrees, width, then the rows (atomic order) sorted ascending
    if (hipMemsetAsync(icnt, 0, sizeof(int) * ns, L.stream) != hipSuccess) return -1;
    MPH_LAUNCH("sinit_transpose", L.stream, k_sinit_transpose, g, b, 0, L.stream, ns, ocnt, *eo, w, icnt,
               (int*)nullptr, 0, 0);
    if (hipMemcpyAsync(h.data(), icnt, sizeof(int) * ns, hipMemcpyDeviceToHost, L.stream) != hipSuccess ||
        hipStreamSynchronize(L.stream) != hipSuccess)
        return -1;
    int wi2 = 1;
    for (int v : h) wi2 = v > wi2 ? v : wi2;
    *ei = (int*)alloc(actx, ntile * wi2 * 64 * sizeof(int));
    if (!*ei) return -3;
    if (hipMemsetAsync(*ei, 0, ntile * wi2 * 64 * sizeof(int), L.stream) != hipSuccess) return -1;
    if (hipMemsetAsync(icnt, 0, sizeof(int) * ns, L.stream) != hipSuccess) return -1;
    MPH_LAUNCH("sinit_transpose", L.stream, k_sinit_transpose, g, b, 0, L.stream, ns, ocnt, *eo, w, icnt, *ei,
               wi2, 1);
    MPH_LAUNCH("sinit_sort_rows", L.stream, k_sinit_sort_rows, g, b, 0, L.stream, ns, icnt, *ei, wi2);
    *wi = wi2;
    if (P.dim == 3)
        MPH_LAUNCH("sinit_normalizer", L.stream, k_sinit_normalizer<3>, g, b, 0, L.stream, P, ns, x0, ocnt, *eo, w,
                   Lm, wx0);
    else
        MPH_LAUNCH("sinit_normalizer", L.stream, k_sinit_normalizer<2>, g, b, 0, L.stream, P, ns, x0, ocnt, *eo, w,
                   Lm, wx0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

void launch_struct_pack(const Launch& L, const double4* src, int w, const int* idx, int m, double4* buf)
{
    Profiler* prof = L.prof;
    if (m <= 0) return;
    MPH_LAUNCH("struct_pack", L.stream, k_struct_pack, dim3(blocks(m * w, 256)), dim3(256), 0, L.stream, src, w,
               idx, m, buf);
}

void launch_struct_unpack(const Launch& L, const double4* buf, int w, const int* idx, int m, double4* dst)
{
    Profiler* prof = L.prof;
    if (m <= 0) return;
    MPH_LAUNCH("struct_unpack", L.stream, k_struct_unpack, dim3(blocks(m * w, 256)), dim3(256), 0, L.stream, buf,
               w, idx, m, dst);
}

void launch_scan(int* cnt, int ncell, int* bsum, int* start, int total, hipStream_t stream, Profiler* prof)
{
    const int nb = blocks(ncell, kScanBlock);
    const int top = nb <= kScanFusedTop;
    MPH_LAUNCH("scan_reduce", stream, k_scan_reduce, dim3(nb), dim3(kScanThreads), 0, stream, cnt, ncell, bsum);
    if (!top)
        MPH_LAUNCH("scan_top", stream, k_scan_top, dim3(1), dim3(1024), 0, stream, bsum, nb);
    MPH_LAUNCH("scan_down", stream, k_scan_down, dim3(nb), dim3(kScanThreads), 0, stream, cnt, ncell, bsum,
               start, total, (const int*)nullptr, top);
}

int dist_blocks(int n) { return blocks(n > 0 ? n : 1, 256); }

void launch_dist_classify(const Launch& L, const SlabGeom& g, int cap, const DistLayout* lay, int move, int* cls,
                          int* bcnt, const int* wface)
{
    Profiler* prof = L.prof;
    const int nb = dist_blocks(cap);
    MPH_LAUNCH("dist_classify", L.stream, k_dist_classify, dim3(nb), dim3(256), 0, L.stream, *L.P, L.st, g,
               L.B, lay, move, cls, bcnt, nb, wface);
}

void launch_dist_early_classify(const Launch& L, const SlabGeom& g, int cap, const DistLayout* lay,
                                const int* wface, int* cls, int* bcnt)
{
    Profiler* prof = L.prof;
    const int nb = dist_blocks(cap);
    MPH_LAUNCH("dist_early_classify", L.stream, k_dist_early_classify, dim3(nb), dim3(256), 0, L.stream, *L.P,
               L.st, g, L.B, lay, wface, cls, bcnt, nb);
}

void launch_dist_early_pack(const Launch& L, int cap, DistLayout* lay, const int* cls, const int* boff, int cap_l,
                            int cap_r, char* buf_l, char* buf_r)
{
    Profiler* prof = L.prof;
    const int nb = dist_blocks(cap);
    MPH_LAUNCH("dist_early_pack", L.stream, k_dist_early_pack, dim3(nb), dim3(256), 0, L.stream, L.B, lay, cls,
               boff, nb, cap_l, cap_r, L.st, buf_l, buf_r);
}

void launch_dist_scatter(const Launch& L, int cap, DistLayout* lay, const int* cls, const int* boff,
                         const Soa& C, int* dseg, int* vidx)
{
    Profiler* prof = L.prof;
    const int nb = dist_blocks(cap);
    MPH_LAUNCH("dist_scatter", L.stream, k_dist_scatter, dim3(nb), dim3(256), 0, L.stream, L.B, lay, cls, boff,
               nb, C, dseg, vidx);
}

void launch_dist_pack(const Launch& L, const Soa& C, DistLayout* lay, int cap_l, int cap_r, char* buf_l,
                      char* buf_r, const VSrc& vs)
{
    Profiler* prof = L.prof;
    MPH_LAUNCH("dist_pack", L.stream, k_dist_pack, dim3(dist_blocks(std::max(cap_l, cap_r)), 2), dim3(256), 0,
               L.stream, C, lay, cap_l, cap_r, L.st, buf_l, buf_r, vs);
}

void launch_dist_unpack(const Launch& L, const char* buf_l, const char* buf_r, DistLayout* lay, int cap_l,
                        int cap_r, int cap, const Soa& C)
{
    Profiler* prof = L.prof;
    MPH_LAUNCH("dist_unpack", L.stream, k_dist_unpack, dim3(dist_blocks(std::max(cap_l, cap_r)), 2), dim3(256), 0,
               L.stream, buf_l, buf_r, lay, cap_l, cap_r, cap, L.st, C);
}

void launch_halo_pack(const Launch& L, const int* dst_of, const DistLayout* lay, int cap_l, int cap_r,
                      const HaloFields& F, double* buf_l, double* buf_r)
{
    Profiler* prof = L.prof;
    MPH_LAUNCH("halo_pack", L.stream, k_halo_pack, dim3(dist_blocks(std::max(cap_l, cap_r)), 2), dim3(256), 0,
               L.stream, dst_of, lay, cap_l, cap_r, F, buf_l, buf_r);
}

void launch_halo_unpack(const Launch& L, const double* buf_l, const double* buf_r, const int* dst_of,
                        const DistLayout* lay, int cap_l, int cap_r, const HaloFields& F)
{
    Profiler* prof = L.prof;
    MPH_LAUNCH("halo_unpack", L.stream, k_halo_unpack, dim3(dist_blocks(std::max(cap_l, cap_r)), 2), dim3(256), 0,
               L.stream, buf_l, buf_r, dst_of, lay, cap_l, cap_r, F);
}

}  // namespace mph
