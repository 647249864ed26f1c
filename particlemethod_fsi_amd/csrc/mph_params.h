// mph_params.h -- plain-old-data structures shared by the host layer (mph_host.cpp) and the
// HIP kernels (mph_kernels.hip).  No HIP types here, so the host files build with g++/hipcc alike.
#pragma once
#include <cmath>

#include <cstddef>
#include <cstdint>

#include "../../include/mph_gpu.h"


namespace mph {

constexpr int kTypes = MPH_TYPE_COUNT;
constexpr int kMaxNeighbor = MPH_MAX_NEIGHBOR_COUNT;
constexpr int kTile = 64;  // ELL neighbour-list tile = one wavefront of i-particles
// Aligned rows (round 6): at the end of a stencil group the search may move
// every lane of a wave on to the wave's highest row, so that the lanes write (and the passes read)
// the rows of the next group together however far their per-column counts drifted apart.  The
// rows a lane skips are gaps; they all lie below kAlignRows (a wave jumps only while its highest
// row is below it), so a lane's list is its rows [0, end) minus at most kMaxJumps gaps, and from
// kAlignRows on it is contiguous.  A tile therefore holds kMaxNeighbor + kAlignRows rows.
constexpr int kAlignRows = 128;
constexpr int kMaxJumps = 6;   // one per interior stencil group end (7 groups)
#ifndef MPH_TILE_EXTRA
#define MPH_TILE_EXTRA kAlignRows   // (A/B diagnostics only: the tile's rows past kMaxNeighbor)
#endif
constexpr int kTileRows = kMaxNeighbor + MPH_TILE_EXTRA;
// Ints from one wave's list tile to the next: kTileRows rows of 64, plus MPH_TILE_PAD rows, so
// that the tiles do not all start on the same power-of-two boundary.  One row: the search 3-4 %
// faster at rest and in the developed flow (five same-box rounds; 4 and 9 rows no faster; the
// list's write-backs unchanged), steps within noise (profiles/r05/tile_pad/)
#ifndef MPH_TILE_PAD
#define MPH_TILE_PAD 1
#endif
constexpr int kTileStride = kTile * (kTileRows + MPH_TILE_PAD);
// Slot of entry k of lane `lane` in its wave's tile (ints): entry k of the 64 lanes in one 256-byte
// row, [k][lane].  (Entries in pairs or fours side by side, rows per half-wave and rows spread by the
// last step's NeighborCount were measured in round 5 and rejected: DESIGN.md section 3.3.)
#if defined(__HIPCC__)
__host__ __device__
#endif
constexpr inline int ell_slot(int k, int lane)
{
    return (k << 6) | lane;
}
// Stencil reach along the contiguous axis: cells there are >= rc / kContigReach wide, and a
// column is the one index range of +-kContigReach cells (thin cells only sharpen the cutoff
// trimming of each column)
#ifndef MPH_SA
#define MPH_SA 2   // rc/2 cells along the contiguous axis (D1M scans 0.048 -> 0.036 ms; rc/3: search -0.006 ms)
#endif
constexpr int kContigReach = MPH_SA;
// Stencil reach across the two outer (column) axes: cells there are >= rc / kReach wide, so a
// +-kReach stencil of (2 kReach + 1)^2 columns covers the acceptance sphere.  kReach = 3 makes the
// cells (rc / 3 = 0.87 dx at RadiusRatio 2.5) narrower than the lattice spacing, so a cell row
// holds one lattice line and a wavefront is a run along that line: the 64 lanes' k-th neighbours
// are then consecutive particles of one neighbour row (coherent gathers in the list passes).
#ifndef MPH_R
#define MPH_R 3
#endif
constexpr int kReach = MPH_R;
constexpr int kGroups = 2 * kReach + 1;   // stencil columns per axis across the column axes
// ELL list entry = sorted index | (type << kTypeShift): pass A reads the neighbour's type with
// its index instead of gathering it (requires fewer than 2^28 particles per context)
constexpr int kTypeShift = 28;
// The list passes gather through buffer descriptors with 32-bit byte offsets; a row without an
// entry of the lane takes this offset, past every record, so the hardware returns zeros without a
// memory access (no cache lookup)
constexpr unsigned kGatherOob = 0xFFFFFFC0u;
constexpr int kIndexMask = (1 << kTypeShift) - 1;
constexpr int kPad = 8;         // extra elements behind every per-particle array (vector over-reads)

inline bool is_fluid(int t) { return t >= 0 && t < 2; }   // main.cpp:69-70
inline bool is_struct(int t) { return t >= 2 && t < 4; }  // main.cpp:71-72
inline bool is_wall(int t) { return t >= 4 && t < 6; }    // main.cpp:73-74

// Axis of the 3-D cell order DevParams.perm at position k (0 slowest, 2 contiguous):
// 0 (x, y, z); for z slabs 1 (z, x, y), 2 (z, y, x), 3 (y, z, x), 4 (x, z, y)
inline constexpr int order_axis(int perm, int k)
{
    return perm == 1 ? (k == 0 ? 2 : k == 1 ? 0 : 1)
         : perm == 2 ? (k == 0 ? 2 : k == 1 ? 1 : 0)
         : perm == 3 ? (k == 0 ? 1 : k == 1 ? 2 : 0)
         : perm == 4 ? (k == 0 ? 0 : k == 1 ? 2 : 1)
                     : k;
}
// the contiguous (half-width-cell) axis of the cell order
inline constexpr int contig_axis(int dim, int perm) { return dim == 2 ? 1 : order_axis(perm, 2); }

// Every constant the reference derives in initializeWeight/Fluid/Wall/Domain
// (main.cpp:1191-1469), in the reference's own arithmetic, plus what the GPU path precomputes.
// Passed by value as a kernel argument (kernarg segment -> scalar loads).
struct DevParams {
    int n;             // particles held by this context (slab mode: the array capacity, a bound)
    // slab mode: the device-resident particle count (DistLayout.n), which the kernels read so
    // that a step needs no host round trip for sizes; null on a single GPU (n is exact)
    const int* n_dev;
    int dim;           // 2 or 3
    int module;        // MphModule
    int wall_motion;   // MphWallMotion
    int surface;      // any CofA != 0 -> surface-tension terms live (K12/K13)
    int n_struct;      // structure particles (types 2,3)
    int gc[3];         // GPU linked-cell grid (gc[2] == 1 in 2-D)
    int ncell;         // gc[0]*gc[1]*gc[2]
    int substeps;      // (int)(Dt/Elastic_Dt + 0.5), main.cpp:653
    int sa;            // stencil half-width (cells) along the contiguous axis (kContigReach)
    // linear order of the 3-D cell grid (order_axis above): 0 = (x, y, z) with z contiguous; z
    // slabs (mph_dist.hip) put z in the middle, 3 = (y, z, x) or 4 = (x, z, y), so that the ghosts
    // beyond both faces form long runs at the two ends of every plane of the slowest axis (whole
    // wavefronts the list kernels skip) while every XCD's contiguous share of the sorted arrays
    // stays a band of that slowest axis through the whole slab (L2 locality); 1, 2 put z slowest
    int perm;
    int fast_ok;       // every active axis has > 12 GPU cells: interior waves may skip the
                       // periodic branch of the minimum image (see k_neighbors)
    double inner_lo[3], inner_hi[3];   // interior box: >= 3 GPU cells from every periodic face
    // the search's interior box in grid offsets (position - corg, wrapped into [0, dw)): >= 3
    // cells from the grid's faces.  The grid origin corg may sit inside an empty band of the
    // domain (choose_grid_origin), so particles at a periodic face of the domain can be interior
    // to the grid; their waves then need the face box above only while particles lie within it at
    // both ends of that axis (DevState.seam_occ) or on the slab axis (seam_always bit)
    double sinner_lo[3], sinner_hi[3];
    int seam_always;
    double dmin[3], dw[3], hw[3], w075[3];   // domain min / width / half width / 0.75 width
    double corg[3];    // origin of the GPU cell grid (dmin, or the slab window's lower edge)
    double ginv[3];    // 1 / GPU cell width per axis
    // slab mode: particles within slab_h of a slab face may have ghost neighbours (pass B runs
    // them after the halo exchange); slab_axis = -1 outside slab mode
    int slab_axis;
    double slab_lo, slab_hi, slab_h;
    double rc2;        // (MaxRadius + MARGIN)^2, main.cpp:1765
    double ra, rg, rp, rv;                   // radii (main.cpp:1195-1198)
    double ra2, rg2, rp2, rv2;               // radius*radius as the reference compares them
    double inv_ra, inv_rg, inv_rp, inv_rv;
    // kernel prefactors: wa = ca*t*(1-t)^2, dwa = cda*(1-t)*(1-3t), w_x = c_x*(1-t)^2,
    // dw_x = cd_x*(1-t)  with t = r/h (main.cpp:298-368)
    double ca, cda, cg, cdg, cp, cdp, cv, cdv;
    double cw;          // weight(): (1/Swp)/rp^dim (main.cpp:268-295)
    double n0a, n0p, r2g, cofk, dx, vol, dt, edt, cvis;
    double cw_pair;    // (1/Swp)(1/RadiusP^dim) of weight() for the elastic pairs (main.cpp:268-295)
    double gravity[3];
    double ratio[kTypes][kTypes];   // InteractionRatio
    double mu_ij[kTypes][kTypes];   // 2 mu_i mu_j / (mu_i + mu_j) from ShearViscosity
    double cofa[kTypes];            // CofA (main.cpp:1339-1341)
    double mass[kTypes], inv_mass[kTypes], density[kTypes], inv_density[kTypes];
    double bulk[kTypes], bulk_visc[kTypes];
    double wall_rot[kTypes][3][3];  // initializeWall (main.cpp:1371-1410)
    double wall_omega[kTypes][3];
    double wall_vel[kTypes][3];
    // Uniform FP64 constants the kernels would otherwise derive per lane (gfx9 has no scalar FP64
    // ALU: a value computed on the device occupies a VGPR pair for the whole loop it is hoisted
    // out of; from the kernel arguments it stays in SGPRs).  set_uniforms fills them.
    double rc2_lo, rc2_hi;   // rc2 (1 - 1e-10), rc2 (1 + 1e-10): the search's exact-test band
    double rc2_trim;         // rc2 (1 + 4e-6): the column-trimming bound
    double cwid[3];          // 1 / ginv: GPU cell widths
    double rg_r2g;           // rg / r2g (GravityCenter, DiffuseInterface)
    double cref[3];          // the domain centre the search's FP32 records are taken from
    float rc2f_lo, rc2f_hi;  // below lo the FP32 r^2 accepts, above hi it rejects (FP64 between)
    // The search stores a neighbour in the list only if its FP32 r^2 <= rlf: the largest radius of
    // the passes' sums (MaxRadius, main.cpp:1199) squared, widened by the FP32 records' error band,
    // so the list holds every pair any sum can take (the passes' exact tests decide) and not the
    // shell MaxRadius < r <= MaxRadius + MARGIN that the reference's list carries and NeighborCount
    // counts.  FLT_MAX (MPH_LIST_FULL=1): the reference's whole list.
    float rlf;
};

// Derived uniforms of DevParams (same expressions the kernels used, so the same bits).
inline void set_uniforms(DevParams& P)
{
    P.rc2_lo = P.rc2 * (1.0 - 1e-10);
    P.rc2_hi = P.rc2 * (1.0 + 1e-10);
    P.rc2_trim = P.rc2 * (1.0 + 4e-6);
    for (int d = 0; d < 3; ++d) P.cwid[d] = 1.0 / P.ginv[d];
    P.rg_r2g = P.rg / P.r2g;
    // FP32 records (the search's): coordinates within half a domain width of the centre, each
    // rounded once (<= 2^-24 x that); a difference is off by <= 2^-23 hw, r^2 near the cutoff by
    // <= 2 sqrt(3) 2^-23 hw / rc relative plus the FP32 sum's few ulp: the band is twice that
    double hwm = 0.0;
    for (int d = 0; d < 3; ++d) {
        P.cref[d] = P.dmin[d] + P.hw[d];
        hwm = P.hw[d] > hwm ? P.hw[d] : hwm;
    }
    const double rc = std::sqrt(P.rc2);
    const double delta = 2.0 * (2.0 * 1.7320508 * hwm * 1.1920929e-7 / rc) + 4.0e-6;
    P.rc2f_lo = (float)(P.rc2 * (1.0 - delta));
    P.rc2f_hi = (float)(P.rc2 * (1.0 + delta));
    const double rmax = std::fmax(std::fmax(P.ra, P.rg), std::fmax(P.rp, P.rv));
    P.rlf = (float)(rmax * rmax * (1.0 + delta));
}

// work histogram of the XCD map: waves in 4096 equal runs (D16M: ~60 waves per run, so the
// search's per-wave atomics spread over ~100 addresses at a time; 512 runs cost its search 7 %)
constexpr int kXcdSegs = 4096;

// Mutable per-step device scalars (so a captured hipGraph can replay many steps).
struct DevState {
    double time;                 // Time
    double wall_c[kTypes][3];    // WallCenter (advanced by V*Dt every step, main.cpp:3066-3070)
    double wall_vel[kTypes][3];  // WallVelocity
    double wall_omega[kTypes][3];// WallOmega
    double wall_rot[kTypes][3][3];  // WallRotation (initializeWall)
    int overflow;                // error bits: 1 neighbour overflow (> MAX_NEIGHBOR_COUNT),
                                 // 2 slab jump (mph_dist), 4 non-finite position, 8 message
                                 // capacity (mph_dist), 64 inconsistent cell histogram
    int pad0;
    // particles within the face box margin of a periodic face, per axis (bit 2k: low face, 2k+1:
    // high face), gathered by k_prep into seam_occ[seam_step & 1]; k_place clears the other word
    // and advances seam_step, so the search reads seam_occ[(seam_step - 1) & 1]
    int seam_occ[2];
    int seam_step;
    int seam_pad;
    // work-balanced XCD map of the two list passes (mph_kernels.hip, list_block): the search adds
    // each wave's work (its longest list + a fixed cost) into seg_work[its 1/kXcdSegs of the waves];
    // the next step's k_rank_scatter turns that into the XCDs' contiguous block ranges (xcd_frac:
    // fractions of 2^16, 0 ... 65536) for the passes and clears seg_work
    int seg_work[kXcdSegs];
    int xcd_frac[9];
    int xcd_pad[3];
};
// the part of DevState the host reads back after steps (the error bits and the step scalars)
constexpr size_t kStateHead = offsetof(DevState, seg_work);

#if defined(__HIPCC__)
#define MPH_HD __host__ __device__
#else
#define MPH_HD
#endif

// Pass A's single-cutoff form (pass_a_term<.., true>) when RadiusA = RadiusP = RadiusV (RadiusG =
// RadiusA, main.cpp:1195-1198), as in every BASELINE config.
#ifndef MPH_PA_EQR
#define MPH_PA_EQR 1
#endif
MPH_HD inline bool pass_a_equal_radii(const DevParams& P)
{
    return MPH_PA_EQR && P.ra == P.rp && P.rv == P.rp && P.rg == P.rp;
}

// Slab decomposition along one axis (multi-GPU, mph_dist.hip).  Rank r owns the particles whose
// (periodically wrapped) coordinate c satisfies lo <= c < hi, with the first/last rank also
// owning any roundoff spill below dmin / above dmax.  `h` is the halo width (>= the neighbour
// cutoff): owned particles within h of a face are mirrored to that neighbour as ghosts.
struct SlabGeom {
    int axis;
    int first, last, lfirst, llast, rfirst, rlast;   // first/last-rank flags: me, left, right
    double lo, hi, llo, lhi, rlo, rhi;               // slabs of me and my periodic neighbours
    double h;
    // elastic-solid particles are owned by the slab of their InitialPosition for good (their
    // fixed Lagrangian lists then never change rank); w = domain width along the axis, smargin =
    // how far beyond a face such a particle may be displaced (h includes it)
    double w, smargin;
};

// Particle classes of one step's redistribution, in the order of their segment in the local
// arrays: [migrate right | band right | inner | band left | migrate left]; kSlabDrop marks ghosts
// of the previous step, kSlabLost a particle that jumped past a neighbour's slab.
enum SlabClass { kMigR = 0, kBandR = 1, kInner = 2, kBandL = 3, kMigL = 4, kSlabDrop = 5,
                 kSlabClasses = 6, kSlabLost = 7 };

MPH_HD inline bool slab_owns(double c, double lo, double hi, int first, int last)
{
    return (first || c >= lo) && (last || c < hi);
}

MPH_HD inline int slab_class(const SlabGeom& g, double c)
{
    if (slab_owns(c, g.lo, g.hi, g.first, g.last)) {
        if (c - g.lo < g.h) return kBandL;
        if (g.hi - c <= g.h) return kBandR;
        return kInner;
    }
    if (slab_owns(c, g.llo, g.lhi, g.lfirst, g.llast)) return kMigL;
    if (slab_owns(c, g.rlo, g.rhi, g.rfirst, g.rlast)) return kMigR;
    return kSlabLost;
}

// Elastic-solid particle of this rank (never migrates): band by its periodic distance from the
// faces, lost if displaced more than smargin beyond one.
MPH_HD inline int slab_class_static(const SlabGeom& g, double c)
{
    const double half = 0.5 * (g.hi - g.lo);
    double off = c - (g.lo + half);
    off -= g.w * __builtin_floor(off / g.w + 0.5);
    const double dl = off + half, dr = half - off;
    if (dl < -g.smargin || dr < -g.smargin) return kSlabLost;
    if (dl < g.h) return kBandL;
    if (dr <= g.h) return kBandR;
    return kInner;
}

// Device-resident sizes of one slab redistribution (mph_dist.hip), written by the kernels of the
// step itself, so that a whole step -- RCCL calls included -- can be captured into a hipGraph.
// send/recv double as the count messages of the exchange (2 ints to each neighbour).
struct DistLayout {
    int n;                        // local particles (owned + ghosts) after the last redistribution
    int n_own;
    int seg[kSlabClasses + 1];    // class segment starts in C (k_dist_scatter)
    int send[4];                  // to the left {bandL, migL}, to the right {migR, bandR}
    int recv[4];                  // from the left their {migR, bandR}, from the right their {bandL, migL}
    int hw[5];                    // high-water marks since the last reset: send_l, send_r, recv_l,
                                  // recv_r, n (capacity tuning between step batches)
    int pad;
};

// Per-type tables read with per-lane type indices (device memory; staged through LDS where hot).
struct DevTables {
    double ratio[kTypes * kTypes];   // InteractionRatio[ti][tj]
    double mu_ij[kTypes * kTypes];   // 2 mu_i mu_j / (mu_i + mu_j)
    double cofa[kTypes], mass[kTypes], inv_mass[kTypes], bulk[kTypes], bulk_visc[kTypes];
};

// Host-side derived constants (reference arithmetic, bit-identical to the reference's globals).
struct HostDerived {
    double ra, rg, rp, rv, max_radius;
    double swa, swg, swp, swv, n0a, n0p, r2g, cofk, cofa[kTypes];
    double vol, dx;
    double dmin[3], dmax[3], dw[3];
    double cell_w;
    int cell_n[3];
    double wall_rot[kTypes][3][3];
};

}  // namespace mph
