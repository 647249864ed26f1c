// mph_kernels.h -- launch interface of the HIP kernels (mph_kernels.hip) used by mph_ctx.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "mph_params.h"

namespace mph {

// Device arrays of the elastic solid, in structure-slot order (see StructureInit).  The fixed
// Lagrangian lists are stored ELL-tiled like the fluid list: entry k of slot s at
// [(s >> 6) * W + k][s & 63], so the 64 lanes of a wavefront read entry k with one coalesced load.
struct StructDev {
    int* orig = nullptr;          // slot -> original particle index
    int* slot_of = nullptr;       // original particle index -> slot (-1: not structure / not owned)
    int* bidx = nullptr;          // slot -> index of its B entry this step (written by pass B)
    int n_own = 0;                // slots computed here (slab mode: owned, then ghost slots)
    // slab mode: the owned slots [0, n_inner) have no ghost slot in their out- or in-list (their
    // substep halves run while the ghost exchange travels); [n_inner, n_own) have one
    int n_inner = 0;
    int wo = 0, wi = 0;           // ELL widths (max out / in count)
    int* ocnt = nullptr;          // InitialStructureNeighborCount per slot
    int* icnt = nullptr;          // in-degree (how many slots list s)
    int* eo_nb = nullptr;         // out-list neighbour slots, ELL [ntile * wo][64]
    int* ei_nb = nullptr;         // in-list (senders i of the reference's scatter), ELL [ntile * wi][64]
    double4* wx0 = nullptr;       // sum_j w_sj x0_sj (the P_s half of StressForce, fixed)
    double* L = nullptr;          // Normalizer [ns][9]
    double2* lame = nullptr;      // (LambdaLames, MuLames)
    double* inv_rho = nullptr;    // 1/Density[type]
    int* clamp = nullptr;         // 0 free, 1 clamped + force zeroed, 2 clamped
    double4* x0 = nullptr;        // InitialPosition
    double4* x = nullptr;         // current position (valid during the substeps)
    double4* v = nullptr;
    double4* u = nullptr;         // displacement Mod(x - x0) (main.cpp:2700-2712), per substep
    double4* P = nullptr;         // first Piola-Kirchhoff F S L: 2-D one double4 {P00,P01,P10,P11}, 3-D 3 rows
    // DeformGradient, Strain, Stress: nine planes each, element 3a + b of slot s at [(3a + b) fes + s]
    double* F = nullptr;
    double* E = nullptr;
    double* S = nullptr;
    int fes = 0;                  // their plane stride (slots allocated)
};

// Per-kernel HIP event timing (mph_profile_steps); nullptr in normal runs.  `events` hands out a
// start/stop pair for one launch and says how to set them: true, from the dispatch packet's own
// timestamps (hipExtLaunchKernelGGL); false, recorded on the stream around the launch.
struct Profiler {
    virtual bool events(const char* name, hipStream_t s, hipEvent_t* start, hipEvent_t* stop) = 0;
    // `waiting` is about to wait for an event `from` has just recorded: the next launch on
    // `waiting` starts no earlier than `from` reaches this point (mph_profile_steps)
    virtual void join(hipStream_t waiting, hipStream_t from) { (void)waiting; (void)from; }
    virtual ~Profiler() = default;
};

// Persistent particle state, one FP64 array per component (structure of arrays): in the
// neighbour loops consecutive lanes gather consecutive elements, so one 8-byte load per lane
// touches ~8-10 cache lines per wavefront instead of ~40 for 32-byte records.
struct Soa {
    double *x = nullptr, *y = nullptr, *z = nullptr;
    double *vx = nullptr, *vy = nullptr, *vz = nullptr;
    int *type = nullptr, *id = nullptr;
    // gather record of the sorted set A (null for B/C): {x, y, z, vx, vy, vz}, 48 bytes, read
    // with three 16-byte loads.  The neighbour loops are bound by the texture-address/data path
    // (profiles/r01: TA ~64 % busy in pass A); the type of j travels in the list entry instead
    // (kTypeShift), so a neighbour costs 48 gathered bytes instead of 64.
    double2* p6 = nullptr;
    // {x, y, z} - domain centre in FP32 and the type's bits, 16 bytes, the search's staged
    // candidate records (sorted set A only)
    float4* f4 = nullptr;
};

// Slab mode: the kept part [0, *n) of the redistributed set C is not copied -- entry v lives in
// the integrated set V at idx[v] (-1 - q: a migrant leaving as a ghost, its id negated on read);
// only the received tail [*n, ...) is in C itself.  idx null: C holds everything (single context).
struct VSrc {
    const int* idx = nullptr;
    const int* n = nullptr;
    Soa V;
};

// Pass B hands the integrated structure particles straight to the slot-ordered elastic arrays
// (null slot_of: no structure particles) and records where each slot's B entry lives (bidx), so
// the last substep can write the result back.
struct StructHook {
    const int* slot_of;
    double4 *sx, *sv, *su;
    const double4* sx0;
    int* bidx;
};

// Everything one launch sequence needs.
struct Launch {
    const DevParams* P = nullptr;
    const DevTables* T = nullptr;
    DevState* st = nullptr;
    hipStream_t stream = nullptr;
    Profiler* prof = nullptr;
    // B set: integrated state in the previous order; A set: cell-sorted current order
    Soa A, B;
    int* rank_of = nullptr;
    int* dst_of = nullptr;        // slab mode: pre-sort index -> sorted index (else rank_of[id])
    int *key = nullptr, *slot = nullptr, *tmp = nullptr, *cnt = nullptr, *start = nullptr, *bsum = nullptr;
    // ncount: each list's rows (what the passes walk); nbcount: NeighborCount (every neighbour within
    // the search radius; the lists keep only r^2 <= DevParams.rlf)
    int *nbr = nullptr, *ncount = nullptr, *nbcount = nullptr;
    // the row jumps of the lists (mph_kernels.hip RowMask): one header word per wave, one word of gap
    // starts per particle; ncount counts rows, gaps included
    unsigned long long *lhdr = nullptr, *lgap = nullptr;
    int* wface = nullptr;         // slab mode: face-wavefront flags written by pass B (early send)
    VSrc vsrc;                    // slab mode: where the sort finds the kept entries of its input
    // fewest particles for the work-balanced XCD map of the passes (split in k_rank_scatter);
    // MPH_XCD_BAL_MIN overrides it at creation (tests force the map on small cases)
    int xcd_bal_min = 1 << 20;
    // pass A products (A order): pressure values, gravity centre (GC, PressureA), sums
    double *pres = nullptr, *gx = nullptr, *gy = nullptr, *gz = nullptr, *pa = nullptr;
    double *dens_a = nullptr, *vstrain = nullptr, *divp = nullptr;
    double4 *fpart = nullptr;   // pass A: P_i half of the pressure force + viscous force
    double4 *rec = nullptr;     // pass A: {x, y, z, PressureP}, the pass-B gather record
    double4 *force = nullptr, *acc = nullptr;   // outputs (A order)
    const StructDev* S = nullptr;
};

void launch_sort(const Launch& L, int mode);   // mode 0 init, 1 step, 2 step (motion done)
void launch_neighbors(const Launch& L);
void launch_pass_a(const Launch& L);
// launch_neighbors + launch_pass_a
void launch_search_pass_a(const Launch& L);
void launch_pass_b(const Launch& L, int phase = 0);   // phase: 0 all, 1/2 slab inner/near-face
void launch_structure(const Launch& L, bool last);   // last: the batch's last step (output tensors)
// calculateInitialNeighbor + calculateNormalizer of the ns structure slots (x0 in slot order) on
// the device: counts (ocnt), ELL out-rows (*eo, width *wo) and their transpose (*ei, *wi), both
// sorted ascending, Normalizer (Lm [ns][9]) and sum_j w_sj x0_sj (wx0).  The ELL arrays are
// allocated through alloc(actx, bytes) once their widths are known.  key/slot/tmp/sorted: ns
// ints of scratch each.  Returns 0, -1 (HIP error), -2 (a slot reached 512 neighbours), -3 (OOM).
int launch_struct_init(const Launch& L, int ns, const double4* x0, int* key, int* slot, int* tmp, int* sorted,
                       int* ocnt, int* icnt, int** eo, int* wo, int** ei, int* wi, double* Lm, double4* wx0,
                       void* (*alloc)(void*, size_t), void* actx);
// over the slots [s0, s1) (s1 < 0: every computed slot, [0, n_own))
// store: also write the output-only tensors F, E, S (the last substep of a batch's last step)
void launch_struct_stress(const Launch& L, bool store, int s0 = 0, int s1 = -1);
void launch_struct_velocity(const Launch& L, bool last, int s0 = 0, int s1 = -1);
// slab mode: rows of per-slot double4 records (w per slot) gathered into / scattered from a message
void launch_struct_pack(const Launch& L, const double4* src, int w, const int* idx, int m, double4* buf);
void launch_struct_unpack(const Launch& L, const double4* buf, int w, const int* idx, int m, double4* dst);
void launch_virial(const Launch& L, const Soa& X, double* vir, double* vpres);   // X: state in A order

// slab decomposition (mph_dist.hip)
struct HaloFields {
    double* f[5];
    int nf;
    double4* rec;   // f[0] (PressureP) is also the P of the pass-B record (its plane stride rec_stride)
    int rec_stride;
};
void launch_scan(int* cnt, int ncell, int* bsum, int* start, int total, hipStream_t stream, Profiler* prof);
int dist_blocks(int n);
// slab redistribution; every size is read from the device layout (graph-capturable).  cap = local
// array capacity, cap_msg = capacity (particles) of the message of that side.
void launch_dist_classify(const Launch& L, const SlabGeom& g, int cap, const DistLayout* lay, int move, int* cls,
                          int* bcnt, const int* wface = nullptr);
void launch_dist_early_classify(const Launch& L, const SlabGeom& g, int cap, const DistLayout* lay,
                                const int* wface, int* cls, int* bcnt);
void launch_dist_early_pack(const Launch& L, int cap, DistLayout* lay, const int* cls, const int* boff, int cap_l,
                            int cap_r, char* buf_l, char* buf_r);
// vidx non-null: record the B index of every kept entry (VSrc) instead of copying it into C
void launch_dist_scatter(const Launch& L, int cap, DistLayout* lay, const int* cls, const int* boff,
                         const Soa& C, int* dseg, int* vidx = nullptr);
// both sides / directions in one launch each (blockIdx.y)
void launch_dist_pack(const Launch& L, const Soa& C, DistLayout* lay, int cap_l, int cap_r, char* buf_l,
                      char* buf_r, const VSrc& vs = VSrc{});
void launch_dist_unpack(const Launch& L, const char* buf_l, const char* buf_r, DistLayout* lay, int cap_l,
                        int cap_r, int cap, const Soa& C);
void launch_halo_pack(const Launch& L, const int* dst_of, const DistLayout* lay, int cap_l, int cap_r,
                      const HaloFields& F, double* buf_l, double* buf_r);
void launch_halo_unpack(const Launch& L, const double* buf_l, const double* buf_r, const int* dst_of,
                        const DistLayout* lay, int cap_l, int cap_r, const HaloFields& F);

}  // namespace mph
