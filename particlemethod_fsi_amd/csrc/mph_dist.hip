// mph_dist.hip -- multi-GPU slab decomposition of the hot path (one process per GPU, RCCL).
//
// The reference has no domain decomposition (one OpenMP/OpenACC process, main.cpp:597-686).  The
// update of a particle depends only on neighbours within the cutoff rc = MaxRadius + MARGIN
// (main.cpp:1765), so the periodic domain is cut into `nranks` slabs along one axis (equal widths,
// or the cuts of MphSlabOptions).  Each rank holds
//
//   owned   particles inside its slab [lo, hi)                (computed, returned by mph_get)
//   ghosts  copies of the neighbours' particles within h >= rc of a face, and of its own
//           particles that crossed a face this step (now owned next door)
//
// One step (this file, dist_step), all on the context's stream:
//
//   1. k_dist_classify: wall motion + periodic wrap (calculateWall / calculatePeriodicBoundary
//      exactly as the single-GPU k_prep), then the slab class of every owned particle; ghosts of
//      the previous step are dropped.
//   2. stable partition into C = [migR | bandR | inner | bandL | migL]     (scan + scatter)
//   3. exchange: to the left neighbour [bandL | migL], to the right [migR | bandR] (56 B per
//      particle, behind a header with the two class counts); received messages are appended to C:
//      [.. | from left: their migR (ours now), their bandR (ghosts) | from right: their bandL
//      (ghosts), their migL (ours now)].  Our own migrants stay in C as ghosts.
//   4. cell sort of C (owned + ghosts) into A, neighbour search, pass A -- the single-GPU kernels
//      on the local window grid (DevParams.corg / gc along the slab axis).
//   5. halo exchange of the pass-A values every neighbour's ghosts need in pass B: PressureP
//      (+ GravityCenter, PressureA with surface tension), 8 or 40 B per ghost.
//   6. pass B (forces, kick, drift) into B.
//
// Owned particles see every neighbour (band width h >= rc), run the same FP64 expressions as
// the single-GPU path, and get bit-identical neighbour sets; sums may be ordered differently
// (local cell grid), so values agree with the single-GPU run to reassociation roundoff.
//
// Elastic-solid particles (types 2, 3) are owned by the slab of their InitialPosition for good:
// their fixed Lagrangian lists (calculateInitialNeighbor, main.cpp:1497-1658) then map to a static
// set of ghost slots owned by the two neighbours (dist_struct_setup).  They never migrate; they
// are mirrored as fluid-pass ghosts like any particle near a face, and may sit up to kStructMargin
// beyond their slab's face (the band width grows by that much).  Each elastic substep
// (main.cpp:653-660) becomes
//   7. ghost displacements u -> k_struct_stress on the owned slots -> ghost stresses P ->
//      k_struct_velocity on the owned slots (the last substep writes the owned B entries).
// Transport: RCCL ncclSend/ncclRecv (xGMI) or a host callback (tests, mph_create_dist_host).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <string>
#include <vector>

#include "mph_ctx.h"

using namespace mph;

namespace {

constexpr size_t kMsgBytes = 56;   // per particle, k_dist_pack layout
constexpr size_t kMsgHead = 16;    // message header: the two class counts
constexpr double kStructMargin = 4.0;   // x ParticleSpacing: elastic particle displacement across a face

#define RCCL_OK(ctx, expr)                                                                     \
    do {                                                                                       \
        ncclResult_t _r = (expr);                                                              \
        if (_r != ncclSuccess)                                                                 \
            return ctx_fail(ctx, MPH_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

// Slab of `rank` along `axis`: equal widths, or the caller's cuts (nranks - 1 interior
// coordinates, ascending; MphSlabOptions.cuts); hi(r) and lo(r+1) are the same expression.
void slab_of(const HostDerived& h, int axis, int rank, int nranks, const double* cuts, double& lo, double& hi)
{
    const double W = h.dw[axis];
    if (cuts) {
        lo = rank == 0 ? h.dmin[axis] : cuts[rank - 1];
        hi = rank == nranks - 1 ? h.dmax[axis] : cuts[rank];
        return;
    }
    lo = rank == 0 ? h.dmin[axis] : h.dmin[axis] + W * rank / nranks;
    hi = rank == nranks - 1 ? h.dmax[axis] : h.dmin[axis] + W * (rank + 1) / nranks;
}

// cuts strictly ascending inside the domain (NULL: equal widths)
int check_cuts(const HostDerived& h, int axis, int nranks, const double* cuts, std::string& err)
{
    if (!cuts) return MPH_OK;
    for (int k = 0; k < nranks - 1; ++k) {
        const double lo = k == 0 ? h.dmin[axis] : cuts[k - 1];
        if (!(cuts[k] > lo) || !(cuts[k] < h.dmax[axis])) {
            err = "slab cuts must ascend strictly inside the domain";
            return MPH_ERR_ARG;
        }
    }
    return MPH_OK;
}

const double* dist_cuts(const MphDist& D) { return D.cuts.empty() ? nullptr : D.cuts.data(); }

SlabGeom make_geom(const HostDerived& h, int axis, int rank, int nranks, const double* cuts, double halo)
{
    SlabGeom g{};
    g.axis = axis;
    g.w = h.dw[axis];
    const int l = (rank + nranks - 1) % nranks, r = (rank + 1) % nranks;
    slab_of(h, axis, rank, nranks, cuts, g.lo, g.hi);
    slab_of(h, axis, l, nranks, cuts, g.llo, g.lhi);
    slab_of(h, axis, r, nranks, cuts, g.rlo, g.rhi);
    g.first = rank == 0; g.last = rank == nranks - 1;
    g.lfirst = l == 0; g.llast = l == nranks - 1;
    g.rfirst = r == 0; g.rlast = r == nranks - 1;
    g.h = halo;
    return g;
}

double wrap_coord(const HostDerived& h, int axis, double x)
{
#pragma clang fp contract(off)
    const double w = h.dw[axis];
    const double u = x - h.dmin[axis];
    return u - w * std::floor(u / w) + h.dmin[axis];
}

double halo_width(const DevParams& P) { return std::sqrt(P.rc2) * (1.0 + 1e-6); }

int owner_rank(const HostDerived& h, int axis, int nranks, const double* cuts, double x)
{
    const double a = wrap_coord(h, axis, x);
    for (int r = 0; r < nranks; ++r) {
        double lo, hi;
        slab_of(h, axis, r, nranks, cuts, lo, hi);
        if (slab_owns(a, lo, hi, r == 0, r == nranks - 1)) return r;
    }
    return nranks - 1;
}

// signed periodic offset of x from the centre of rank r's slab
double slab_offset(const HostDerived& h, int axis, int r, int nranks, const double* cuts, double x)
{
    double lo, hi;
    slab_of(h, axis, r, nranks, cuts, lo, hi);
    const double W = h.dw[axis];
    double off = x - 0.5 * (lo + hi);
    off -= W * std::floor(off / W + 0.5);
    return off;
}

int check_geometry(const MphConfig& cfg, int nranks, int axis, std::string& err)
{
    if (nranks < 2) { err = "slab mode needs nranks >= 2 (use mph_create)"; return MPH_ERR_ARG; }
    if (axis < 0 || axis > 2 || (cfg.dim == 2 && axis == 2)) { err = "invalid slab axis"; return MPH_ERR_ARG; }
    return MPH_OK;
}

int copy_soa(MphCtx* c, const Soa& dst, const Soa& src, int n)
{
    double* dd[6] = {dst.x, dst.y, dst.z, dst.vx, dst.vy, dst.vz};
    const double* sd[6] = {src.x, src.y, src.z, src.vx, src.vy, src.vz};
    for (int k = 0; k < 6; ++k)
        MPH_HIP_OK(c, hipMemcpyAsync(dd[k], sd[k], sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
    MPH_HIP_OK(c, hipMemcpyAsync(dst.type, src.type, sizeof(int) * n, hipMemcpyDeviceToDevice, c->stream));
    MPH_HIP_OK(c, hipMemcpyAsync(dst.id, src.id, sizeof(int) * n, hipMemcpyDeviceToDevice, c->stream));
    return MPH_OK;
}

// -- transport ----------------------------------------------------------------------------------

// send_l -> left neighbour (arrives there as its recv_r), send_r -> right neighbour (its recv_l)
int exchange(MphCtx* c, hipStream_t stream, const void* send_l, size_t bsl, const void* send_r, size_t bsr,
             void* recv_l, size_t brl, void* recv_r, size_t brr)
{
    MphDist& D = *c->dist;
    if (D.rccl) {
        ncclComm_t comm = (ncclComm_t)D.comm;
        RCCL_OK(c, ncclGroupStart());
        // per-peer order: first the left-going message, then the right-going one (matters when
        // left == right, nranks == 2): a rank's first receive from a peer matches that peer's
        // first send, i.e. its left-going message = our from-right message
        if (bsl) RCCL_OK(c, ncclSend(send_l, bsl, ncclChar, D.left, comm, stream));
        if (brr) RCCL_OK(c, ncclRecv(recv_r, brr, ncclChar, D.right, comm, stream));
        if (bsr) RCCL_OK(c, ncclSend(send_r, bsr, ncclChar, D.right, comm, stream));
        if (brl) RCCL_OK(c, ncclRecv(recv_l, brl, ncclChar, D.left, comm, stream));
        RCCL_OK(c, ncclGroupEnd());
        return MPH_OK;
    }
    const size_t region = D.region;
    if (bsl > region || bsr > region || brl > region || brr > region)
        return ctx_fail(c, MPH_ERR_CAPACITY, "slab mode: message larger than the staging buffers");
    char* hs_l = D.host_stage;
    char* hs_r = D.host_stage + region;
    char* hr_l = D.host_stage + 2 * region;
    char* hr_r = D.host_stage + 3 * region;
    // the previous exchange's host-to-device copies may still read the receive halves (when it ran
    // on the other stream, this stream's synchronisation below does not cover them)
    if (D.stage_busy) MPH_HIP_OK(c, hipEventSynchronize(D.ev_stage));
    if (bsl) MPH_HIP_OK(c, hipMemcpyAsync(hs_l, send_l, bsl, hipMemcpyDeviceToHost, stream));
    if (bsr) MPH_HIP_OK(c, hipMemcpyAsync(hs_r, send_r, bsr, hipMemcpyDeviceToHost, stream));
    MPH_HIP_OK(c, hipStreamSynchronize(stream));
    if (D.host_fn(D.host_user, hs_l, bsl, hs_r, bsr, hr_l, brl, hr_r, brr) != 0)
        return ctx_fail(c, MPH_ERR_TRANSPORT, "host exchange callback failed");
    if (brl) MPH_HIP_OK(c, hipMemcpyAsync(recv_l, hr_l, brl, hipMemcpyHostToDevice, stream));
    if (brr) MPH_HIP_OK(c, hipMemcpyAsync(recv_r, hr_r, brr, hipMemcpyHostToDevice, stream));
    if (!D.ev_stage) MPH_HIP_OK(c, hipEventCreateWithFlags(&D.ev_stage, hipEventDisableTiming));
    MPH_HIP_OK(c, hipEventRecord(D.ev_stage, stream));
    D.stage_busy = true;
    return MPH_OK;
}

template <typename T>
T* lay_field(DistLayout* lay, size_t off) { return reinterpret_cast<T*>(reinterpret_cast<char*>(lay) + off); }

// Message capacity (particles) of a direction whose live count is c: 25 % + 4096 particles of room
// to grow before the next capacity check (dist_sync, at most kSyncSteps steps later).  The slack
// can be lowered (MPH_SLAB_MSG_SLACK, tests of the growth path); both ranks of a pair read the same
// environment, so they still derive equal capacities for their shared direction.
int msg_slack()
{
    static const int s = [] {
        const char* e = std::getenv("MPH_SLAB_MSG_SLACK");
        return e ? std::max(0, std::atoi(e)) : 4096;
    }();
    return s;
}
int msg_capacity(int c);

// MPH_SLAB_MSG_CAP0_FRAC: the first sizing (mph_create) gives frac x the counts and no slack, so
// the first capacity check grows them (tests of the growth path)
int msg_capacity0(int c)
{
    static const double frac = [] {
        const char* e = std::getenv("MPH_SLAB_MSG_CAP0_FRAC");
        return e ? std::atof(e) : 0.0;
    }();
    return frac > 0.0 ? std::max(1, (int)std::ceil(frac * c)) : msg_capacity(c);
}

int msg_capacity(int c)
{
    // MPH_SLAB_MSG_CAP: one fixed capacity for every direction (tests of the overflow report)
    static const int fixed = [] {
        const char* e = std::getenv("MPH_SLAB_MSG_CAP");
        return e ? std::max(0, std::atoi(e)) : 0;
    }();
    return fixed > 0 ? fixed : c + c / 4 + msg_slack();
}

// Steps between two capacity checks inside one mph_step call: a long call (the steps between two
// VTK outputs) must not outrun its message capacities while the flow changes, so dist_step
// replays at most this many steps before dist_sync reads the high-water marks and grows them.
constexpr int kSyncSteps = 32;

// (Re)allocate the four message buffers for the current capacities: redistribution (56 B per
// particle), pass-A halo (up to 40 B per particle of both directions' capacities), elastic ghosts.
int msg_alloc(MphCtx* c)
{
    MphDist& D = *c->dist;
    const size_t most = std::max({D.cap_sl, D.cap_sr, D.cap_rl, D.cap_rr});
    size_t region = kMsgHead + kMsgBytes * most;
    region = std::max(region, sizeof(double) * 5 * (size_t)std::max(D.cap_sl + D.cap_rl, D.cap_sr + D.cap_rr));
    const size_t smost = std::max({D.nss_l, D.nss_r, D.nsr_l, D.nsr_r});
    region = std::max(region, 3 * sizeof(double4) * smost);
    region = (region + 255) & ~(size_t)255;
    if (region <= D.region && D.send_l) return MPH_OK;
    for (char** b : {&D.send_l, &D.send_r, &D.recv_l, &D.recv_r}) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
        MPH_HIP_OK(c, hipMalloc((void**)b, region));
    }
    if (!D.rccl) {
        if (D.stage_busy) MPH_HIP_OK(c, hipEventSynchronize(D.ev_stage));   // no copy still reads it
        D.stage_busy = false;
        if (D.host_stage) (void)hipHostFree(D.host_stage);
        D.host_stage = nullptr;
        MPH_HIP_OK(c, hipHostMalloc((void**)&D.host_stage, 4 * region, hipHostMallocDefault));
    }
    D.region = region;
    return MPH_OK;
}

// a cross-stream wait for an event `from` has just recorded (the profiler keeps the point as the
// earliest start of the next launch on `waiting`, see EventProfiler)
hipError_t stream_wait(Profiler* prof, hipStream_t waiting, hipEvent_t ev, hipStream_t from)
{
    if (prof) prof->join(waiting, from);
    return hipStreamWaitEvent(waiting, ev, 0);
}

// the redistributed set's kept entries: where they live in B (VSrc, D.virt) or nowhere (in C)
VSrc dist_vsrc(MphCtx* c)
{
    MphDist& D = *c->dist;
    VSrc vs;
    if (D.virt) {
        vs.idx = D.vidx;
        vs.n = lay_field<int>(D.lay, offsetof(DistLayout, seg)) + kSlabDrop;
        vs.V = c->L.B;
    }
    return vs;
}

// Steps 1-3 of the protocol: classify, partition, exchange migrants + ghosts.  Leaves the new
// local set (owned and ghosts) in D.C and its sizes in D.lay -- on the device: nothing here reads
// a size on the host, so the step can be captured.  init: first redistribution of mph_create,
// which reads the counts once to size the message buffers.
// early_in: the messages left at the end of the previous step (early_send); here only the local
// partition, then the wait for them and the unpack
int redistribute(MphCtx* c, bool move, bool init, Profiler* prof, bool early_in = false)
{
    MphDist& D = *c->dist;
    Launch L = c->L;
    L.prof = prof;
    const int nb = dist_blocks(D.cap);
    // see early_send (no profiler floor: the second stream has moved on to the exchange since)
    if (early_in) MPH_HIP_OK(c, hipStreamWaitEvent(c->stream, D.ev_s, 0));
    launch_dist_classify(L, D.g, D.cap, D.lay, move ? 1 : 0, D.cls, D.bcnt, early_in ? D.wface : nullptr);
    launch_scan(D.bcnt, kSlabClasses * nb, D.bsum, D.boff, 0, c->stream, prof);
    launch_dist_scatter(L, D.cap, D.lay, D.cls, D.boff, D.C, lay_field<int>(D.lay, offsetof(DistLayout, seg)),
                        D.virt ? D.vidx : nullptr);
    if (early_in) {
        MPH_HIP_OK(c, stream_wait(prof, c->stream, D.ev_x, D.stream2));
        launch_dist_unpack(L, D.recv_l, D.recv_r, D.lay, D.cap_rl, D.cap_rr, D.cap, D.C);
        return MPH_OK;
    }
    if (init) {
        // the first redistribution exchanges the counts alone, to size the message buffers; later
        // ones find them in the message headers (one exchange per redistribution)
        int* snd = lay_field<int>(D.lay, offsetof(DistLayout, send));
        int* rcv = lay_field<int>(D.lay, offsetof(DistLayout, recv));
        MPH_CK(exchange(c, c->stream, snd, 2 * sizeof(int), snd + 2, 2 * sizeof(int), rcv, 2 * sizeof(int),
                        rcv + 2, 2 * sizeof(int)));
        MPH_HIP_OK(c, hipMemcpyAsync(D.hlay, D.lay, sizeof(DistLayout), hipMemcpyDeviceToHost, c->stream));
        MPH_HIP_OK(c, hipStreamSynchronize(c->stream));
        const DistLayout& h = *D.hlay;
        D.cap_sl = msg_capacity0(h.send[0] + h.send[1]);
        D.cap_sr = msg_capacity0(h.send[2] + h.send[3]);
        D.cap_rl = msg_capacity0(h.recv[0] + h.recv[1]);
        D.cap_rr = msg_capacity0(h.recv[2] + h.recv[3]);
        MPH_CK(msg_alloc(c));
    }
    const VSrc vs = dist_vsrc(c);
    launch_dist_pack(L, D.C, D.lay, D.cap_sl, D.cap_sr, D.send_l, D.send_r, vs);
    MPH_CK(exchange(c, c->stream, D.send_l, kMsgHead + kMsgBytes * D.cap_sl, D.send_r,
                    kMsgHead + kMsgBytes * D.cap_sr, D.recv_l, kMsgHead + kMsgBytes * D.cap_rl, D.recv_r,
                    kMsgHead + kMsgBytes * D.cap_rr));
    launch_dist_unpack(L, D.recv_l, D.recv_r, D.lay, D.cap_rl, D.cap_rr, D.cap, D.C);
    return MPH_OK;
}

// The next step's redistribution messages, sent from the face wavefronts of this step's pass B
// on the second stream (joined by the next step's redistribute(early_in)); the same bytes as
// k_dist_pack would send from C.
int early_send(MphCtx* c, Profiler* prof, hipStream_t stream)
{
    MphDist& D = *c->dist;
    Launch L = c->L;
    L.prof = prof;
    L.stream = stream;
    const int nb = dist_blocks(D.cap);
    launch_dist_early_classify(L, D.g, D.cap, D.lay, D.wface, D.cls, D.bcnt);
    launch_scan(D.bcnt, kSlabClasses * nb, D.bsum, D.boff, 0, stream, prof);
    launch_dist_early_pack(L, D.cap, D.lay, D.cls, D.boff, D.cap_sl, D.cap_sr, D.send_l, D.send_r);
    // ev_s: the face waves' pass B and these kernels are done (the next step's partition, on the
    // main stream, waits for it before it reads B and wface); ev_x: the messages have landed
    MPH_HIP_OK(c, hipEventRecord(D.ev_s, stream));
    if (stream != D.stream2) MPH_HIP_OK(c, stream_wait(prof, D.stream2, D.ev_s, stream));
    MPH_CK(exchange(c, D.stream2, D.send_l, kMsgHead + kMsgBytes * D.cap_sl, D.send_r,
                    kMsgHead + kMsgBytes * D.cap_sr, D.recv_l, kMsgHead + kMsgBytes * D.cap_rl, D.recv_r,
                    kMsgHead + kMsgBytes * D.cap_rr));
    MPH_HIP_OK(c, hipEventRecord(D.ev_x, D.stream2));
    return MPH_OK;
}

// cell sort of C into A (slab-local grid), recording dst_of = pre-sort -> sorted index
void sort_local(MphCtx* c, int mode, Profiler* prof)
{
    Launch L = c->L;
    L.prof = prof;
    L.B = c->dist->C;
    L.vsrc = dist_vsrc(c);
    L.dst_of = c->rank_of;
    launch_sort(L, mode);
}

HaloFields halo_fields(MphCtx* c)
{
    HaloFields F{};
    F.f[0] = c->pres;
    F.nf = 1;
    F.rec = c->rec;
    F.rec_stride = c->P.n;   // the plane stride of the pass-B records (capacity)
    if (c->P.surface) {
        F.f[1] = c->gx; F.f[2] = c->gy; F.f[3] = c->gz; F.f[4] = c->pa;
        F.nf = 5;
    }
    return F;
}

// Step 5: the pass-A values of every neighbour's ghosts (ranges from the device layout, fixed
// message capacities: to/from the left cap_sl + cap_rl particles, to/from the right cap_sr + cap_rr).
int halo_exchange(MphCtx* c, Profiler* prof, hipStream_t stream, const HaloFields* fields = nullptr)
{
    MphDist& D = *c->dist;
    Launch L = c->L;
    L.prof = prof;
    L.stream = stream;
    const HaloFields F = fields ? *fields : halo_fields(c);
    const int capl = D.cap_sl + D.cap_rl, capr = D.cap_sr + D.cap_rr;
    double* sl = (double*)D.send_l;
    double* sr = (double*)D.send_r;
    double* rl = (double*)D.recv_l;
    double* rr = (double*)D.recv_r;
    launch_halo_pack(L, c->rank_of, D.lay, capl, capr, F, sl, sr);
    const size_t b = sizeof(double) * F.nf;
    MPH_CK(exchange(c, stream, sl, b * capl, sr, b * capr, rl, b * capl, rr, b * capr));
    launch_halo_unpack(L, rl, rr, c->rank_of, D.lay, capl, capr, F);
    return MPH_OK;
}

// One static ghost exchange of per-slot double4 records (w rows per slot) of the elastic arrays.
int struct_exchange(MphCtx* c, double4* a, int w, Profiler* prof, hipStream_t stream)
{
    MphDist& D = *c->dist;
    Launch L = c->L;
    L.prof = prof;
    L.stream = stream;
    double4* sl = (double4*)D.send_l;
    double4* sr = (double4*)D.send_r;
    double4* rl = (double4*)D.recv_l;
    double4* rr = (double4*)D.recv_r;
    launch_struct_pack(L, a, w, D.ss_l, D.nss_l, sl);
    launch_struct_pack(L, a, w, D.ss_r, D.nss_r, sr);
    const size_t b = sizeof(double4) * w;
    MPH_CK(exchange(c, stream, sl, b * D.nss_l, sr, b * D.nss_r, rl, b * D.nsr_l, rr, b * D.nsr_r));
    launch_struct_unpack(L, rl, w, D.sr_l, D.nsr_l, a);
    launch_struct_unpack(L, rr, w, D.sr_r, D.nsr_r, a);
    return MPH_OK;
}

// Step 7: the elastic substeps on the owned slots, ghosts refreshed before each half.  Each ghost
// exchange (displacements u before DeformationVector/Stress, first Piola-Kirchhoff rows P before
// StressForce) travels on the second stream while the owned slots whose lists hold no ghost slot
// ([0, n_inner), dist_struct_setup) run their half on the main stream; the others follow once it
// has landed.  The slots a neighbour needs are all among the latter (symmetric lists), so a pack
// never waits for an inner half.
int struct_substeps(MphCtx* c, Profiler* prof)
{
    if (c->P.n_struct == 0) return MPH_OK;
    MphDist& D = *c->dist;
    Launch L = c->L;
    L.prof = prof;
    StructDev& S = c->Sd;
    const int wP = c->P.dim == 2 ? 1 : 3;
    // launch(s0, s1): the half-substep over owned slots [s0, s1)
    auto half = [&](double4* a, int w, auto&& launch) -> int {
        if (!D.overlap) {
            MPH_CK(struct_exchange(c, a, w, prof, c->stream));
            launch(0, S.n_own);
            return MPH_OK;
        }
        MPH_HIP_OK(c, hipEventRecord(D.ev_a, c->stream));
        MPH_HIP_OK(c, stream_wait(prof, D.stream2, D.ev_a, c->stream));
        launch(0, S.n_inner);   // enqueued before a host-staged exchange blocks the host
        MPH_CK(struct_exchange(c, a, w, prof, D.stream2));
        MPH_HIP_OK(c, hipEventRecord(D.ev_h, D.stream2));
        MPH_HIP_OK(c, stream_wait(prof, c->stream, D.ev_h, D.stream2));
        launch(S.n_inner, S.n_own);
        return MPH_OK;
    };
    for (int sub = 0; sub < c->P.substeps; ++sub) {
        const bool last = sub == c->P.substeps - 1;
        MPH_CK(half(S.u, 1, [&](int s0, int s1) { launch_struct_stress(L, last, s0, s1); }));
        MPH_CK(half(S.P, wP, [&](int s0, int s1) { launch_struct_velocity(L, last, s0, s1); }));
    }
    return MPH_OK;
}

// Element-wise max of v[0..n) over all ranks (every rank ends with the same values): RCCL
// all-reduce, or n-1 rounds along the ring of the host transport (each passes its running max left).
int collective_max(MphCtx* c, double* v, int n)
{
    MphDist& D = *c->dist;
    if (D.rccl) {
        double* d = nullptr;
        MPH_HIP_OK(c, hipMalloc((void**)&d, sizeof(double) * n));
        std::unique_ptr<double, void (*)(double*)> guard(d, [](double* q) { (void)hipFree(q); });
        MPH_HIP_OK(c, hipMemcpyAsync(d, v, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
        RCCL_OK(c, ncclAllReduce(d, d, n, ncclDouble, ncclMax, (ncclComm_t)D.comm, c->stream));
        MPH_HIP_OK(c, hipMemcpyAsync(v, d, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
        MPH_HIP_OK(c, hipStreamSynchronize(c->stream));
        return MPH_OK;
    }
    std::vector<double> in((size_t)n);
    for (int round = 1; round < D.nranks; ++round) {
        if (D.host_fn(D.host_user, v, sizeof(double) * n, nullptr, 0, nullptr, 0, in.data(), sizeof(double) * n) != 0)
            return ctx_fail(c, MPH_ERR_TRANSPORT, "host exchange callback failed (collective max)");
        for (int k = 0; k < n; ++k) v[k] = std::max(v[k], in[k]);
    }
    return MPH_OK;
}

// MPH_SLAB_OVERLAP unset ("auto"): the ranks choose the pass-B mode together at creation, from
// what this machine and transport do.  On the initial state (after the init sums) every rank times,
// with events on its stream, best of three after a warm-up:
//   th  the halo exchange of the pass-A values,
//   tr  an exchange of the redistribution messages,
//   ts  pass B as the overlap splits it (interior, then face waves) minus pass B in one launch;
// the maxima over ranks decide: overlap when th + tr > ts, i.e. when the exchanges it can hide
// behind the interior pass B (and, with the early send, behind the next partition) cost more than
// splitting pass B does.  The exchanges are timed at their message capacities, which is what the
// steps send: the messages of a step have fixed, capacity-sized lengths (the live counts travel in
// their headers), so that RCCL steps can be replayed from captured graphs.
// The probe touches no live state: its halo packs from and unpacks into the redistribution
// scratch set C (which every step rewrites before reading, dist_enqueue_step), its redistribution
// exchange moves the message buffers only, and its trial pass B integrates into C with the output
// stores (Force, Acceleration) off.  Every rank takes part or none: a rank holding elastic
// particles (whose pass B also hands them to the substep slots) keeps the overlap off on all ranks,
// agreed through a collective max, since the structure need not reach every slab.
int overlap_probe(MphCtx* c)
{
    MphDist& D = *c->dist;
    D.overlap = D.overlap_mode == 1;
    if (D.overlap_mode >= 0) return MPH_OK;
    double any_struct = c->P.n_struct > 0 ? 1.0 : 0.0;
    MPH_CK(collective_max(c, &any_struct, 1));
    if (any_struct > 0.0) return MPH_OK;
    Launch L = c->L;
    L.wface = D.wface;
    L.B = D.C;                   // the trial pass B's integrated state: scratch
    L.force = L.acc = nullptr;   // no output stores
    HaloFields F = halo_fields(c);
    double* scratch[5] = {D.C.x, D.C.y, D.C.z, D.C.vx, D.C.vy};
    for (int k = 0; k < F.nf; ++k) F.f[k] = scratch[k];
    F.rec = nullptr;
    hipEvent_t e[5] = {};
    struct Ev {
        hipEvent_t* e;
        ~Ev() { for (int k = 0; k < 5; ++k) if (e[k]) (void)hipEventDestroy(e[k]); }
    } guard{e};
    for (auto& x : e) MPH_HIP_OK(c, hipEventCreate(&x));
    double best[3] = {1e30, 1e30, 1e30};
    for (int rep = 0; rep < 4; ++rep) {
        MPH_HIP_OK(c, hipEventRecord(e[0], c->stream));
        MPH_CK(halo_exchange(c, nullptr, c->stream, &F));
        MPH_HIP_OK(c, hipEventRecord(e[1], c->stream));
        MPH_CK(exchange(c, c->stream, D.send_l, kMsgHead + kMsgBytes * D.cap_sl, D.send_r,
                        kMsgHead + kMsgBytes * D.cap_sr, D.recv_l, kMsgHead + kMsgBytes * D.cap_rl, D.recv_r,
                        kMsgHead + kMsgBytes * D.cap_rr));
        MPH_HIP_OK(c, hipEventRecord(e[2], c->stream));
        launch_pass_b(L, 0);
        MPH_HIP_OK(c, hipEventRecord(e[3], c->stream));
        launch_pass_b(L, 1);
        launch_pass_b(L, 2);
        MPH_HIP_OK(c, hipEventRecord(e[4], c->stream));
        MPH_HIP_OK(c, hipGetLastError());
        MPH_HIP_OK(c, hipEventSynchronize(e[4]));
        float ms[4];
        for (int k = 0; k < 4; ++k) MPH_HIP_OK(c, hipEventElapsedTime(&ms[k], e[k], e[k + 1]));
        if (rep == 0) continue;   // warm-up: the first exchanges set up the transport
        best[0] = std::min(best[0], (double)ms[0]);
        best[1] = std::min(best[1], (double)ms[1]);
        best[2] = std::min(best[2], (double)ms[3] - (double)ms[2]);
    }
    MPH_CK(collective_max(c, best, 3));
    for (int k = 0; k < 3; ++k) D.probe_ms[k] = best[k];
    D.overlap = best[0] + best[1] > best[2];
    return MPH_OK;
}

}  // namespace

namespace mph {

int dist_setup(MphCtx* c, const double* pos, std::vector<int>& owned)
{
    MphDist& D = *c->dist;
    const HostDerived& h = c->h;
    const int axis = D.g.axis;
    std::string err;
    MPH_CK(ctx_fail(c, check_geometry(c->cfg, D.nranks, axis, err), err));
    D.left = (D.rank + D.nranks - 1) % D.nranks;
    D.right = (D.rank + 1) % D.nranks;
    // elastic particles may be displaced up to kStructMargin dx beyond their static slab
    const bool has_struct = !c->S.orig.empty();
    const double smargin = has_struct ? kStructMargin * h.dx : 0.0;
    const double halo = halo_width(c->P) + smargin;
    MPH_CK(ctx_fail(c, check_cuts(h, axis, D.nranks, dist_cuts(D), err), err));
    D.g = make_geom(h, axis, D.rank, D.nranks, dist_cuts(D), halo);
    D.g.smargin = smargin;
    const double W = h.dw[axis];
    const double cw = W / c->P.gc[axis];
    // slabs must be wider than two halos plus a migration margin, so that a band particle is
    // mirrored to one neighbour only and a migrant reaches only the adjacent slab
    for (int r = 0; r < D.nranks; ++r) {
        double lo, hi;
        slab_of(h, axis, r, D.nranks, dist_cuts(D), lo, hi);
        if (hi - lo < 2.0 * halo + 2.0 * h.dx)
            return ctx_fail(c, MPH_ERR_DOMAIN, "slab width " + std::to_string(hi - lo) + " below two halo widths (" +
                                                   std::to_string(2.0 * halo) + ")");
    }
    // local window grid along the slab axis: [lo - h - cw, hi + h + cw)
    const double wlo = D.g.lo - halo - cw, whi = D.g.hi + halo + cw;
    const int gloc = (int)std::ceil((whi - wlo) / cw);
    const int m = stencil_margin(c->P, axis);
    if (gloc < 2 * m - 1) return ctx_fail(c, MPH_ERR_DOMAIN, "slab window narrower than the cell stencil");
    c->P.corg[axis] = wlo;
    c->P.slab_axis = axis;
    c->P.slab_lo = D.g.lo;
    c->P.slab_hi = D.g.hi;
    // pass B's face wavefronts (particles within slab_h of a face, integrated after the halo) also
    // carry every particle the next redistribution can send: one step moves a particle far less
    // than the 2 dx margin (checked: k_dist_classify flags a sender outside them)
    c->P.slab_h = halo + 2.0 * h.dx;
    c->P.gc[axis] = std::min(gloc, c->P.gc[axis] + 1);
    // fast-path interior: >= 3 cells inside both the window and the periodic domain
    c->P.inner_lo[axis] = std::max(wlo, h.dmin[axis]) + m * cw * (1.0 + 1e-9);
    c->P.inner_hi[axis] = std::min(whi, h.dmax[axis]) - m * cw * (1.0 + 1e-9);
    // the search's box in offsets from the window's edge; the face box always applies on this axis
    c->P.sinner_lo[axis] = std::max(wlo, h.dmin[axis]) - wlo + m * cw * (1.0 + 1e-9);
    c->P.sinner_hi[axis] = std::min(whi, h.dmax[axis]) - wlo - m * cw * (1.0 + 1e-9);
    c->P.seam_always |= 1 << axis;
    // initial owned set and a capacity for owned + ghosts (+ headroom for migration imbalance)
    owned.clear();
    size_t near = 0;
    const int nin = (int)c->prop.size();   // the particles passed in (all, or this rank's window)
    for (int i = 0; i < nin; ++i) {
        const double a = wrap_coord(h, axis, pos[3 * (size_t)i + axis]);
        if (is_struct(c->prop[i])) {
            // static owner: the slab of the InitialPosition
            if (owner_rank(h, axis, D.nranks, dist_cuts(D), c->pos0[3 * (size_t)i + axis]) == D.rank)
                owned.push_back(i);
            else ++near;
            continue;
        }
        if (slab_owns(a, D.g.lo, D.g.hi, D.g.first, D.g.last)) {
            owned.push_back(i);
        } else {
            // within h + 2 dx outside a face (periodic distance): a ghost candidate
            double dl = D.g.lo - a, dh = a - D.g.hi;
            dl -= W * std::floor(dl / W);
            dh -= W * std::floor(dh / W);
            if (std::min(dl, dh) <= halo + 2.0 * h.dx) ++near;
        }
    }
    const size_t want = (size_t)((owned.size() + near) * 1.25) + 65536;
    D.cap = (int)std::min<size_t>(want, (size_t)c->n_glob);
    D.n_own = (int)owned.size();
    return MPH_OK;
}

int dist_struct_setup(MphCtx* c, std::vector<int>& lsl, int& n_own, int& n_inner)
{
    MphDist& D = *c->dist;
    const HostDerived& h = c->h;
    const StructureInit& S = c->S;
    const int axis = D.g.axis, R = D.nranks;
    const int ns = (int)S.orig.size();
    std::vector<int> owner(ns);
    const double* cuts = dist_cuts(D);
    for (int s = 0; s < ns; ++s) owner[s] = owner_rank(h, axis, R, cuts, c->pos0[3 * (size_t)S.orig[s] + axis]);
    // ghost slots of rank r: the list neighbours (out- and in-lists) of its owned slots that other
    // ranks own, split by side (periodic offset of x0 from r's slab centre), ascending slot id
    std::string err;
    auto ghosts = [&](int r, std::vector<int>& gl, std::vector<int>& gr) {
        std::vector<char> seen(ns, 0);
        gl.clear();
        gr.clear();
        const int left = (r + R - 1) % R, right = (r + 1) % R;
        auto visit = [&](int j) {
            if (owner[j] == r || seen[j]) return;
            seen[j] = 1;
            const bool lside = slab_offset(h, axis, r, R, cuts, c->pos0[3 * (size_t)S.orig[j] + axis]) < 0.0;
            if (owner[j] != (lside ? left : right)) err = "structure list spans more than one slab";
            (lside ? gl : gr).push_back(j);
        };
        for (int s = 0; s < ns; ++s) {
            if (owner[s] != r) continue;
            for (int q = S.offset[s]; q < S.offset[s + 1]; ++q) visit(S.nbr[q]);
            for (int q = S.in_offset[s]; q < S.in_offset[s + 1]; ++q) visit(S.in_nbr[q]);
        }
        std::sort(gl.begin(), gl.end());
        std::sort(gr.begin(), gr.end());
    };
    std::vector<int> gl, gr, lgl, lgr, rgl, rgr;
    ghosts(D.rank, gl, gr);
    ghosts(D.left, lgl, lgr);
    ghosts(D.right, rgl, rgr);
    if (!err.empty()) return ctx_fail(c, MPH_ERR_DOMAIN, "slab mode: " + err);
    // the owned slots, those without a ghost slot in their out- or in-list first (the lists are
    // symmetric, so every slot a neighbour needs is among the others): their substep halves run
    // while the ghost exchange travels (struct_substeps)
    lsl.clear();
    std::vector<int> outer;
    for (int s = 0; s < ns; ++s) {
        if (owner[s] != D.rank) continue;
        bool ghost = false;
        for (int q = S.offset[s]; q < S.offset[s + 1] && !ghost; ++q) ghost = owner[S.nbr[q]] != D.rank;
        for (int q = S.in_offset[s]; q < S.in_offset[s + 1] && !ghost; ++q) ghost = owner[S.in_nbr[q]] != D.rank;
        (ghost ? outer : lsl).push_back(s);
    }
    n_inner = (int)lsl.size();
    lsl.insert(lsl.end(), outer.begin(), outer.end());
    n_own = (int)lsl.size();
    std::vector<int> loc(ns, -1);
    for (int k = 0; k < n_own; ++k) loc[lsl[k]] = k;
    std::vector<int> rl, rr, sl, sr;
    for (int j : gl) { rl.push_back((int)lsl.size()); loc[j] = (int)lsl.size(); lsl.push_back(j); }
    for (int j : gr) { rr.push_back((int)lsl.size()); loc[j] = (int)lsl.size(); lsl.push_back(j); }
    // to the left: the left rank's from-right ghosts (ours); to the right: its from-left ghosts
    for (int j : lgr) sl.push_back(loc[j]);
    for (int j : rgl) sr.push_back(loc[j]);
    for (int k : sl) if (k < 0 || k >= n_own) return ctx_fail(c, MPH_ERR_DOMAIN, "slab mode: elastic ghost routing");
    for (int k : sr) if (k < 0 || k >= n_own) return ctx_fail(c, MPH_ERR_DOMAIN, "slab mode: elastic ghost routing");
    D.nss_l = (int)sl.size(); D.nss_r = (int)sr.size();
    D.nsr_l = (int)rl.size(); D.nsr_r = (int)rr.size();
    MPH_CK(ctx_dalloc(c, &D.ss_l, sl.size())); MPH_CK(ctx_dalloc(c, &D.ss_r, sr.size()));
    MPH_CK(ctx_dalloc(c, &D.sr_l, rl.size())); MPH_CK(ctx_dalloc(c, &D.sr_r, rr.size()));
    auto up = [&](int* d, const std::vector<int>& v) {
        return v.empty() ? hipSuccess : hipMemcpy(d, v.data(), sizeof(int) * v.size(), hipMemcpyHostToDevice);
    };
    MPH_HIP_OK(c, up(D.ss_l, sl)); MPH_HIP_OK(c, up(D.ss_r, sr));
    MPH_HIP_OK(c, up(D.sr_l, rl)); MPH_HIP_OK(c, up(D.sr_r, rr));
    return MPH_OK;
}

int dist_alloc(MphCtx* c)
{
    MphDist& D = *c->dist;
    const int cap = D.cap;
    Soa& C = D.C;
    MPH_CK(ctx_dalloc(c, &C.x, cap)); MPH_CK(ctx_dalloc(c, &C.y, cap)); MPH_CK(ctx_dalloc(c, &C.z, cap));
    MPH_CK(ctx_dalloc(c, &C.vx, cap)); MPH_CK(ctx_dalloc(c, &C.vy, cap)); MPH_CK(ctx_dalloc(c, &C.vz, cap));
    MPH_CK(ctx_dalloc(c, &C.type, cap)); MPH_CK(ctx_dalloc(c, &C.id, cap));
    MPH_CK(ctx_dalloc(c, &D.cls, cap));
    MPH_CK(ctx_dalloc(c, &D.vidx, cap));
    MPH_CK(ctx_dalloc(c, &D.wface, (size_t)cap / 64 + 2));
    MPH_HIP_OK(c, hipMemsetAsync(D.wface, 0, sizeof(int) * ((size_t)cap / 64 + 2), c->stream));
    const size_t nslots = (size_t)kSlabClasses * dist_blocks(cap);
    MPH_CK(ctx_dalloc(c, &D.bcnt, nslots + 1));
    MPH_CK(ctx_dalloc(c, &D.boff, nslots + 1));
    MPH_CK(ctx_dalloc(c, &D.bsum, nslots / 4096 + 2));
    MPH_CK(ctx_dalloc(c, &D.lay, 1));
    MPH_HIP_OK(c, hipHostMalloc((void**)&D.hlay, sizeof(DistLayout), hipHostMallocDefault));
    std::memset(D.hlay, 0, sizeof(DistLayout));
    D.hlay->n = c->n;   // the uploaded owned set, classified by the first redistribution
    MPH_HIP_OK(c, hipMemcpyAsync(D.lay, D.hlay, sizeof(DistLayout), hipMemcpyHostToDevice, c->stream));
    // every kernel of a slab step reads the live particle count from the layout; P.n is the
    // capacity the launch grids are sized for
    c->P.n = cap;
    c->P.n_dev = lay_field<int>(D.lay, offsetof(DistLayout, n));
    // first message buffers (the count exchange of the first redistribution uses them); their
    // capacities follow from the first counts (redistribute, init)
    D.cap_sl = D.cap_sr = D.cap_rl = D.cap_rr = msg_capacity(0);
    MPH_CK(msg_alloc(c));
    MPH_HIP_OK(c, hipStreamCreateWithFlags(&D.stream2, hipStreamNonBlocking));
    MPH_HIP_OK(c, hipEventCreateWithFlags(&D.ev_a, hipEventDisableTiming));
    MPH_HIP_OK(c, hipEventCreateWithFlags(&D.ev_h, hipEventDisableTiming));
    MPH_HIP_OK(c, hipEventCreateWithFlags(&D.ev_s, hipEventDisableTiming));
    MPH_HIP_OK(c, hipEventCreateWithFlags(&D.ev_x, hipEventDisableTiming));
    if (D.rccl) {
        ncclUniqueId id;
        std::memcpy(&id, D.uid, sizeof(id));
        ncclComm_t comm = nullptr;
        RCCL_OK(c, ncclCommInitRank(&comm, D.nranks, id, D.rank));
        D.comm = comm;
    }
    return MPH_OK;
}

int dist_sync(MphCtx* c, bool grow_ok)
{
    MphDist& D = *c->dist;
    DevState hs;
    MPH_HIP_OK(c, hipMemcpyAsync(&hs, c->dst, kStateHead, hipMemcpyDeviceToHost, c->stream));
    MPH_HIP_OK(c, hipMemcpyAsync(D.hlay, D.lay, sizeof(DistLayout), hipMemcpyDeviceToHost, c->stream));
    MPH_HIP_OK(c, hipStreamSynchronize(c->stream));
    if (hs.overflow & 8)
        return ctx_fail(c, MPH_ERR_CAPACITY, "slab mode: a redistribution exceeded the message or local capacity");
    MPH_CK(ctx_state_status(c, hs));
    const DistLayout& h = *D.hlay;
    c->n = h.n;
    D.n_own = h.n_own;
    if (h.hw[4] > D.cap)
        return ctx_fail(c, MPH_ERR_CAPACITY, "slab mode: local particle capacity " + std::to_string(D.cap) +
                                                 " exceeded (" + std::to_string(h.hw[4]) + ")");
    // capacity check between batches: a direction above 90 % of its message capacity grows (both
    // ranks of the pair see the same counts, so they grow the shared direction alike); the
    // captured graphs hold the old sizes and are re-captured by the next step.  Capacities are
    // 1.25 c + 4096: every message travels at its capacity (fixed sizes in the graphs)
    int* caps[4] = {&D.cap_sl, &D.cap_sr, &D.cap_rl, &D.cap_rr};
    bool grow = false;
    for (int k = 0; k < 4 && grow_ok; ++k)
        if ((long long)h.hw[k] * 10 > (long long)*caps[k] * 9) {
            *caps[k] = msg_capacity(h.hw[k]);
            grow = true;
        }
    if (grow) {
        MPH_CK(msg_alloc(c));
        if (c->graph1) { (void)hipGraphExecDestroy(c->graph1); c->graph1 = nullptr; }
        if (c->graph8) { (void)hipGraphExecDestroy(c->graph8); c->graph8 = nullptr; }
        MPH_HIP_OK(c, hipMemsetAsync(lay_field<int>(D.lay, offsetof(DistLayout, hw)), 0, 4 * sizeof(int),
                                     c->stream));
    }
    return MPH_OK;
}

int dist_init(MphCtx* c)
{
    // calculateNeighbor, DensityA, GravityCenter, DensityP of the initialisation (main.cpp:565-568)
    // on owned + ghosts (no motion, no time advance)
    MPH_CK(redistribute(c, false, true, nullptr));
    sort_local(c, 0, nullptr);
    launch_search_pass_a(c->L);
    // no capacity growth yet: the first sizing came from these very counts (and a test sizing,
    // MPH_SLAB_MSG_CAP0_FRAC, is meant to grow at the first check after real steps)
    MPH_CK(dist_sync(c, false));
    // the integrated-state set B starts as the sorted local set (owned + ghosts, ids signed)
    MPH_CK(copy_soa(c, c->B, c->A, c->n));
    MPH_HIP_OK(c, hipGetLastError());
    MPH_CK(dist_sync(c, false));
    MPH_CK(overlap_probe(c));   // MPH_SLAB_OVERLAP auto: the pass-B mode, the same on every rank
    return dist_sync(c, false);
}

// One slab step on the context's stream (no host synchronisation inside: RCCL transport steps
// are captured into graphs by dist_step; the host transport stages each message through host
// memory and so synchronises in exchange()).
// early_in / early_out: inside a batch of steps, this step's redistribution messages were sent by
// the previous step / the next step's are sent here (early_send), beside the interior pass B.
int dist_enqueue_step(MphCtx* c, Profiler* prof, bool early_in, bool early_out)
{
    Launch L = c->L;
    L.prof = prof;
    MphDist& D = *c->dist;
    L.wface = D.wface;
    MPH_CK(redistribute(c, true, false, prof, early_in));
    sort_local(c, 2, prof);
    launch_search_pass_a(L);
    if (!D.overlap) {   // MPH_SLAB_OVERLAP=0: halo first, then one pass B over every particle
        MPH_CK(halo_exchange(c, prof, c->stream));
        launch_pass_b(L, 0);
        if (early_out) MPH_CK(early_send(c, prof, c->stream));
        return struct_substeps(c, prof);
    }
    // pass B of the wavefronts without ghost neighbours runs on the main stream while, on the
    // second stream, the pass-A halo travels and the wavefronts near a face follow as soon as it
    // has landed: the two pass-B kernels run concurrently, so neither launch's tail idles the GPU
    // (the interior one is enqueued first, so that a host-staged exchange, which blocks the host,
    // also overlaps with it).  With the early send the face waves' particles then leave for the
    // next step's redistribution, still on the second stream.
    Launch L2 = L;
    L2.stream = D.stream2;
    MPH_HIP_OK(c, hipEventRecord(D.ev_a, c->stream));
    MPH_HIP_OK(c, stream_wait(prof, D.stream2, D.ev_a, c->stream));
    launch_pass_b(L, 1);
    MPH_CK(halo_exchange(c, prof, D.stream2));
    launch_pass_b(L2, 2);
    // joined by the next step's redistribute (ev_s, ev_x)
    if (early_out && c->P.n_struct == 0) return early_send(c, prof, D.stream2);
    MPH_HIP_OK(c, hipEventRecord(D.ev_h, D.stream2));
    MPH_HIP_OK(c, stream_wait(prof, c->stream, D.ev_h, D.stream2));
    MPH_CK(struct_substeps(c, prof));
    // elastic particles take their positions from the substeps: their face waves are classified
    // and packed after them (main stream); the messages still travel on the second stream beside
    // the next step's partition
    if (early_out) return early_send(c, prof, c->stream);
    return MPH_OK;
}

// the early send chains the steps of one batch (one graph or one mph_step call): step k receives
// early if k > 0 and sends early if k < steps - 1, so every batch ends joined
bool early_at(const MphCtx* c, int k, int steps, int out)
{
    const MphDist& D = *c->dist;
    if (!D.early || !D.overlap) return false;
    return out ? k < steps - 1 : k > 0;
}

int dist_capture(MphCtx* c, int steps, hipGraphExec_t* out)
{
    hipGraph_t g = nullptr;
    MPH_HIP_OK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    int rc = MPH_OK;
    for (int k = 0; k < steps && rc == MPH_OK; ++k) rc = dist_enqueue_step(c, nullptr, early_at(c, k, steps, 0),
                                                                           early_at(c, k, steps, 1));
    const hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (rc != MPH_OK) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    MPH_HIP_OK(c, e);
    const hipError_t ei = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    MPH_HIP_OK(c, ei);
    MPH_HIP_OK(c, hipGraphUpload(*out, c->stream));   // the first launch then costs what later ones do
    return MPH_OK;
}

int dist_step_batch(MphCtx* c, int nsteps, Profiler* prof);

int dist_step(MphCtx* c, int nsteps, Profiler* prof)
{
    // sub-batches of kSyncSteps (a multiple of the 8-step graph), each ending in dist_sync
    for (int done = 0; done < nsteps;) {
        const int k = std::min(kSyncSteps, nsteps - done);
        MPH_CK(dist_step_batch(c, k, prof));
        done += k;
    }
    return MPH_OK;
}

int dist_step_batch(MphCtx* c, int nsteps, Profiler* prof)
{
    MphDist& D = *c->dist;
    int left = nsteps;
    if (D.graphs && !prof) {
        // a capture the runtime refuses (an RCCL build without graph support) falls back to the
        // same steps as direct launches, reported by mph_dist_info
        if (!c->graph1 && dist_capture(c, 1, &c->graph1) != MPH_OK) {
            (void)hipGetLastError();
            D.graphs = false;
            c->err.clear();
            return dist_step_batch(c, nsteps, prof);
        }
        // the 8-step graph at the first call whatever its count (every rank makes the same calls),
        // so a short warm-up does not leave its capture to the first long run
        if (!c->graph8 && dist_capture(c, 8, &c->graph8) != MPH_OK) {
            (void)hipGetLastError();
            D.graphs = false;
            c->err.clear();
            return dist_step_batch(c, nsteps, prof);
        }
        while (left >= 8) { MPH_HIP_OK(c, hipGraphLaunch(c->graph8, c->stream)); left -= 8; }
        while (left > 0) { MPH_HIP_OK(c, hipGraphLaunch(c->graph1, c->stream)); left -= 1; }
    } else {
        for (int k = 0; k < nsteps; ++k)
            MPH_CK(dist_enqueue_step(c, prof, early_at(c, k, nsteps, 0), early_at(c, k, nsteps, 1)));
    }
    MPH_HIP_OK(c, hipGetLastError());
    for (int k = 0; k < nsteps; ++k) c->time += c->cfg.dt;
    c->stepped = true;
    return dist_sync(c);
}

// ---- output in slab mode (collective calls: every rank enters them at the same step) ---------
//
// The reference writes .prof before a step, runs calculateVirialStressAtParticle and writes .vtk
// after one (main.cpp:583-589, 672-683, 957-1189), always for the whole problem.  Here every rank
// packs the records of the particles it owns, rank 0 gathers them (RCCL: one receive from every
// rank; host transport: forwarded along the ring of neighbour exchanges), restores the original
// order and writes the file with the single-context writers, so the bytes are the reference's.

// rank 0 receives the concatenation of every rank's bytes in rank order; the others get nothing
int dist_gather_root(MphCtx* c, const std::vector<char>& mine, std::vector<char>& all)
{
    MphDist& D = *c->dist;
    const int R = D.nranks;
    all.clear();
    if (R == 1) {
        all = mine;
        return MPH_OK;
    }
    if (D.rccl) {
        struct DevBuf {
            void* p = nullptr;
            ~DevBuf() { if (p) (void)hipFree(p); }
        } dsz, dsend, drecv;
        MPH_HIP_OK(c, hipMalloc(&dsz.p, sizeof(long long) * R));
        long long* sz = (long long*)dsz.p;
        const long long my = (long long)mine.size();
        MPH_HIP_OK(c, hipMemcpyAsync(sz + D.rank, &my, sizeof(my), hipMemcpyHostToDevice, c->stream));
        RCCL_OK(c, ncclAllGather(sz + D.rank, sz, 1, ncclInt64, (ncclComm_t)D.comm, c->stream));
        std::vector<long long> h(R);
        MPH_HIP_OK(c, hipMemcpyAsync(h.data(), sz, sizeof(long long) * R, hipMemcpyDeviceToHost, c->stream));
        MPH_HIP_OK(c, hipStreamSynchronize(c->stream));
        long long total = 0;
        std::vector<long long> off(R);
        for (int r = 0; r < R; ++r) { off[r] = total; total += h[r]; }
        if (D.rank != 0 && my > 0) {
            MPH_HIP_OK(c, hipMalloc(&dsend.p, (size_t)my));
            MPH_HIP_OK(c, hipMemcpy(dsend.p, mine.data(), (size_t)my, hipMemcpyHostToDevice));
        }
        if (D.rank == 0 && total > my) MPH_HIP_OK(c, hipMalloc(&drecv.p, (size_t)(total - my)));
        RCCL_OK(c, ncclGroupStart());
        for (int r = 1; r < R; ++r) {
            if (!h[r]) continue;
            if (D.rank == 0)
                RCCL_OK(c, ncclRecv((char*)drecv.p + (off[r] - my), (size_t)h[r], ncclChar, r, (ncclComm_t)D.comm,
                                    c->stream));
            else if (D.rank == r)
                RCCL_OK(c, ncclSend(dsend.p, (size_t)h[r], ncclChar, 0, (ncclComm_t)D.comm, c->stream));
        }
        RCCL_OK(c, ncclGroupEnd());
        MPH_HIP_OK(c, hipStreamSynchronize(c->stream));
        if (D.rank == 0) {
            all.resize((size_t)total);
            std::memcpy(all.data(), mine.data(), mine.size());
            if (total > my)
                MPH_HIP_OK(c, hipMemcpy(all.data() + my, drecv.p, (size_t)(total - my), hipMemcpyDeviceToHost));
        }
        return MPH_OK;
    }
    // host transport: R - 1 rounds along the ring; in round k every rank passes to its left
    // neighbour what it received in round k - 1 (first its own bytes), so rank 0 receives the
    // bytes of rank k in round k
    std::vector<char> carry = D.rank == 0 ? std::vector<char>() : mine;
    if (D.rank == 0) all = mine;
    for (int round = 1; round < R; ++round) {
        long long so = (long long)carry.size(), si = 0;
        if (D.host_fn(D.host_user, &so, sizeof(so), nullptr, 0, nullptr, 0, &si, sizeof(si)) != 0)
            return ctx_fail(c, MPH_ERR_TRANSPORT, "host exchange callback failed (output gather sizes)");
        std::vector<char> in((size_t)si);
        if (D.host_fn(D.host_user, carry.data(), (size_t)so, nullptr, 0, nullptr, 0, in.data(), (size_t)si) != 0)
            return ctx_fail(c, MPH_ERR_TRANSPORT, "host exchange callback failed (output gather)");
        if (D.rank == 0) all.insert(all.end(), in.begin(), in.end());
        else carry.swap(in);
    }
    return MPH_OK;
}

namespace {

// one owned particle of an output gather (original index, and what the writers print)
struct OutRec {
    int id, prop, nc, pad;
    double pos[3], pos0[3], vel[3], acc[3], force[3];
};
// one owned elastic slot: InitialStructureNeighborCount, Stress, Strain
struct OutSlot {
    int id, isnc;
    double S[9], E[9];
};

template <typename T>
int fetch(MphCtx* c, const T* d, std::vector<T>& h, size_t count)
{
    h.resize(count);
    if (count) MPH_HIP_OK(c, hipMemcpyAsync(h.data(), d, sizeof(T) * count, hipMemcpyDeviceToHost, c->stream));
    return MPH_OK;
}

// the records of the particles (and elastic slots) this rank owns, behind two counts
int pack_owned(MphCtx* c, std::vector<char>& buf)
{
    const int n = c->n;
    std::vector<int> id, nc;
    std::vector<double> x, y, z, vx, vy, vz;
    std::vector<double4> f, a;
    MPH_CK(fetch(c, (const int*)c->A.id, id, n));
    MPH_CK(fetch(c, (const int*)c->nbcount, nc, n));
    MPH_CK(fetch(c, (const double*)c->B.x, x, n));
    MPH_CK(fetch(c, (const double*)c->B.y, y, n));
    MPH_CK(fetch(c, (const double*)c->B.z, z, n));
    MPH_CK(fetch(c, (const double*)c->B.vx, vx, n));
    MPH_CK(fetch(c, (const double*)c->B.vy, vy, n));
    MPH_CK(fetch(c, (const double*)c->B.vz, vz, n));
    MPH_CK(fetch(c, (const double4*)c->force, f, n));
    MPH_CK(fetch(c, (const double4*)c->acc, a, n));
    const int ns = c->Sd.n_own;
    std::vector<double> S, E;
    const size_t fes = (size_t)c->Sd.fes;   // nine element planes (StructDev)
    if (ns) {
        MPH_CK(fetch(c, (const double*)c->Sd.S, S, 9 * fes));
        MPH_CK(fetch(c, (const double*)c->Sd.E, E, 9 * fes));
    }
    MPH_HIP_OK(c, hipStreamSynchronize(c->stream));
    std::vector<OutRec> rec;
    rec.reserve((size_t)c->dist->n_own);
    for (int i = 0; i < n; ++i) {
        if (id[i] < 0) continue;   // a ghost
        OutRec r{};
        r.id = id[i];
        // host index of the static inputs (original order, or the slab-local creation's ids)
        const size_t k = c->gid.empty() ? (size_t)id[i]
                                        : (size_t)(std::lower_bound(c->gid.begin(), c->gid.end(), id[i]) - c->gid.begin());
        if (k >= c->prop.size()) return ctx_fail(c, MPH_ERR_ARG, "slab output: an owned particle without static inputs");
        r.prop = c->prop[k];
        r.nc = nc[i];
        const double p[3] = {x[i], y[i], z[i]}, v[3] = {vx[i], vy[i], vz[i]};
        const double ac[3] = {a[i].x, a[i].y, a[i].z}, fo[3] = {f[i].x, f[i].y, f[i].z};
        for (int d = 0; d < 3; ++d) {
            r.pos[d] = p[d];
            r.pos0[d] = c->pos0[3 * k + d];
            r.vel[d] = v[d];
            r.acc[d] = ac[d];
            r.force[d] = fo[d];
        }
        rec.push_back(r);
    }
    std::vector<OutSlot> sl((size_t)ns);
    for (int s = 0; s < ns; ++s) {
        sl[s].id = c->sl_orig[s];
        sl[s].isnc = c->S.count[c->sl_s[s]];
        for (int e = 0; e < 9; ++e) {
            sl[s].S[e] = S[e * fes + s];
            sl[s].E[e] = E[e * fes + s];
        }
    }
    const long long cnt[2] = {(long long)rec.size(), (long long)sl.size()};
    buf.resize(sizeof(cnt) + sizeof(OutRec) * rec.size() + sizeof(OutSlot) * sl.size());
    char* o = buf.data();
    std::memcpy(o, cnt, sizeof(cnt));
    o += sizeof(cnt);
    if (!rec.empty()) std::memcpy(o, rec.data(), sizeof(OutRec) * rec.size());
    o += sizeof(OutRec) * rec.size();
    if (!sl.empty()) std::memcpy(o, sl.data(), sizeof(OutSlot) * sl.size());
    return MPH_OK;
}

// the arrays of the single-context writers, in original order, from every rank's records
struct OutArrays {
    std::vector<int> prop, isnc, nc;
    std::vector<double> pos, pos0, vel, acc, force, stress, strain;
};

int unpack_all(MphCtx* c, const std::vector<char>& all, int nranks, OutArrays& o)
{
    const size_t n = (size_t)c->n_glob;
    o.prop.assign(n, 0); o.isnc.assign(n, 0); o.nc.assign(n, 0);
    o.pos.assign(3 * n, 0.0); o.pos0.assign(3 * n, 0.0); o.vel.assign(3 * n, 0.0);
    o.acc.assign(3 * n, 0.0); o.force.assign(3 * n, 0.0);
    o.stress.assign(9 * n, 0.0); o.strain.assign(9 * n, 0.0);
    std::vector<char> seen(n, 0);
    size_t got = 0;
    const char* p = all.data();
    const char* end = p + all.size();
    for (int r = 0; r < nranks; ++r) {
        long long cnt[2];
        if ((size_t)(end - p) < sizeof(cnt)) return ctx_fail(c, MPH_ERR_TRANSPORT, "slab output: truncated gather");
        std::memcpy(cnt, p, sizeof(cnt));
        p += sizeof(cnt);
        if ((size_t)(end - p) < sizeof(OutRec) * cnt[0] + sizeof(OutSlot) * cnt[1])
            return ctx_fail(c, MPH_ERR_TRANSPORT, "slab output: truncated gather");
        for (long long k = 0; k < cnt[0]; ++k, p += sizeof(OutRec)) {
            OutRec q;
            std::memcpy(&q, p, sizeof(q));
            if (q.id < 0 || (size_t)q.id >= n || seen[q.id])
                return ctx_fail(c, MPH_ERR_CAPACITY, "slab output: ownership is not a partition");
            seen[q.id] = 1;
            ++got;
            const size_t i = (size_t)q.id;
            o.prop[i] = q.prop;
            o.nc[i] = q.nc;
            for (int d = 0; d < 3; ++d) {
                o.pos[3 * i + d] = q.pos[d];
                o.pos0[3 * i + d] = q.pos0[d];
                o.vel[3 * i + d] = q.vel[d];
                o.acc[3 * i + d] = q.acc[d];
                o.force[3 * i + d] = q.force[d];
            }
        }
        for (long long k = 0; k < cnt[1]; ++k, p += sizeof(OutSlot)) {
            OutSlot q;
            std::memcpy(&q, p, sizeof(q));
            if (q.id < 0 || (size_t)q.id >= n) return ctx_fail(c, MPH_ERR_TRANSPORT, "slab output: bad slot record");
            const size_t i = (size_t)q.id;
            o.isnc[i] = q.isnc;
            std::memcpy(&o.stress[9 * i], q.S, sizeof(q.S));
            std::memcpy(&o.strain[9 * i], q.E, sizeof(q.E));
        }
    }
    if (got != n) return ctx_fail(c, MPH_ERR_CAPACITY, "slab output: " + std::to_string(n - got) + " particles owned by no rank");
    return MPH_OK;
}

}  // namespace

int dist_write_output(MphCtx* c, const char* path, int kind)
{
    MphDist& D = *c->dist;
    std::vector<char> mine, all;
    MPH_CK(pack_owned(c, mine));
    MPH_CK(dist_gather_root(c, mine, all));
    mine.clear();
    mine.shrink_to_fit();
    if (D.rank != 0) return MPH_OK;
    auto o = std::make_shared<OutArrays>();
    MPH_CK(unpack_all(c, all, D.nranks, *o));
    all.clear();
    all.shrink_to_fit();
    const int n = c->n_glob;
    if (kind == kOutProf)
        return mph_write_prof_arrays(path, &c->cfg, c->time, n, o->prop.data(), o->pos.data(), o->pos0.data(),
                                     o->vel.data());
    auto write = [o, n](const std::string& pth, bool xml) {
        auto writer = xml ? mph_write_vtu_arrays : mph_write_vtk_arrays;
        return writer(pth.c_str(), n, o->prop.data(), o->pos.data(), o->pos0.data(), o->vel.data(), o->acc.data(),
                      o->force.data(), o->stress.data(), o->strain.data(), o->isnc.data(), o->nc.data());
    };
    if (kind == kOutVtkAsync) {
        const std::string pth = path;
        c->out_thread = std::thread([c, write, pth] { c->out_rc = write(pth, false); });
        return MPH_OK;
    }
    const int rc = write(path, kind == kOutVtu);
    return rc ? ctx_fail(c, rc, std::string("writing ") + path) : MPH_OK;
}

// calculateVirialStressAtParticle (main.cpp:3077-3318) in slab mode: the owned particles' sums need
// their ghost neighbours' post-step positions and velocities, which the owners computed -- one
// halo exchange of B (the pass-A values the virial reads are the particle's own)
int dist_virial(MphCtx* c)
{
    HaloFields F{};
    F.nf = 3;
    F.f[0] = c->B.x; F.f[1] = c->B.y; F.f[2] = c->B.z;
    MPH_CK(halo_exchange(c, nullptr, c->stream, &F));
    F.f[0] = c->B.vx; F.f[1] = c->B.vy; F.f[2] = c->B.vz;
    MPH_CK(halo_exchange(c, nullptr, c->stream, &F));
    MPH_CK(virial_full_lists(c));
    launch_virial(c->L, c->B, c->vir, c->vpres);
    MPH_HIP_OK(c, hipGetLastError());
    MPH_HIP_OK(c, hipStreamSynchronize(c->stream));
    return MPH_OK;
}

void dist_free(MphCtx* c)
{
    MphDist* D = c->dist;
    if (!D) return;
    if (D->stream2) (void)hipStreamSynchronize(D->stream2);
    if (D->comm) (void)ncclCommDestroy((ncclComm_t)D->comm);
    if (D->ev_a) (void)hipEventDestroy(D->ev_a);
    if (D->ev_h) (void)hipEventDestroy(D->ev_h);
    if (D->ev_s) (void)hipEventDestroy(D->ev_s);
    if (D->ev_x) (void)hipEventDestroy(D->ev_x);
    if (D->ev_stage) (void)hipEventDestroy(D->ev_stage);
    if (D->stream2) (void)hipStreamDestroy(D->stream2);
    if (D->hlay) (void)hipHostFree(D->hlay);
    for (char* b : {D->send_l, D->send_r, D->recv_l, D->recv_r})
        if (b) (void)hipFree(b);
    if (D->host_stage) (void)hipHostFree(D->host_stage);
    delete D;
    c->dist = nullptr;
}

}  // namespace mph

extern "C" {

int mph_dist_unique_id(char* out128)
{
    if (!out128) return MPH_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MPH_ERR_RCCL;
    static_assert(sizeof(id) == 128, "ncclUniqueId size");
    std::memcpy(out128, &id, sizeof(id));
    return MPH_OK;
}

int mph_create_dist(MphCtx** ctx, const MphConfig* cfg, int n, const int* property, const double* pos,
                    const double* pos0, const double* vel, int device, int rank, int nranks,
                    const char* unique_id128, int axis)
{
    if (!unique_id128 || rank < 0 || rank >= nranks) return MPH_ERR_ARG;
    MphDist* D = new MphDist();
    D->rank = rank;
    D->nranks = nranks;
    D->g.axis = axis;
    D->rccl = true;
    D->graphs = std::getenv("MPH_SLAB_GRAPHS") == nullptr || std::string(std::getenv("MPH_SLAB_GRAPHS")) != "0";
    std::memcpy(D->uid, unique_id128, sizeof(D->uid));
    return ctx_create(ctx, cfg, n, property, pos, pos0, vel, device, D);
}

int mph_create_slab(MphCtx** ctx, const MphConfig* cfg, int n, const int* property, const double* pos,
                    const double* pos0, const double* vel, int device, const MphSlabOptions* opt)
{
    if (!opt || opt->rank < 0 || opt->rank >= opt->nranks) return MPH_ERR_ARG;
    if ((opt->unique_id128 == nullptr) == (opt->host_fn == nullptr)) return MPH_ERR_ARG;
    if (opt->n_glob > 0 && !opt->ids) return MPH_ERR_ARG;
    MphDist* D = new MphDist();
    D->rank = opt->rank;
    D->nranks = opt->nranks;
    D->g.axis = opt->axis;
    if (opt->cuts) D->cuts.assign(opt->cuts, opt->cuts + std::max(opt->nranks - 1, 0));
    if (opt->unique_id128) {
        D->rccl = true;
        D->graphs = std::getenv("MPH_SLAB_GRAPHS") == nullptr || std::string(std::getenv("MPH_SLAB_GRAPHS")) != "0";
        std::memcpy(D->uid, opt->unique_id128, sizeof(D->uid));
    } else {
        D->host_fn = opt->host_fn;
        D->host_user = opt->host_user;
    }
    return ctx_create(ctx, cfg, n, property, pos, pos0, vel, device, D, opt->n_glob > 0 ? opt->ids : nullptr,
                      opt->n_glob);
}

int mph_create_dist_host(MphCtx** ctx, const MphConfig* cfg, int n, const int* property, const double* pos,
                         const double* pos0, const double* vel, int device, int rank, int nranks, int axis,
                         mph_host_exchange_fn fn, void* user)
{
    if (!fn || rank < 0 || rank >= nranks) return MPH_ERR_ARG;
    MphDist* D = new MphDist();
    D->rank = rank;
    D->nranks = nranks;
    D->g.axis = axis;
    D->host_fn = fn;
    D->host_user = user;
    return ctx_create(ctx, cfg, n, property, pos, pos0, vel, device, D);
}

int mph_dist_selftest(int device)
{
    // one-rank RCCL communicator whose left and right neighbour are itself: exercises the
    // group send/recv of exchange() including the per-peer message order that nranks == 2
    // relies on (our first receive from a peer = its first, left-going, send)
    MphCtx c;
    MphDist* D = new MphDist();
    c.dist = D;
    D->rccl = true;
    D->nranks = 1;
    int status = MPH_OK;
    auto run = [&]() -> int {
        MPH_HIP_OK(&c, hipSetDevice(device));
        MPH_HIP_OK(&c, hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        ncclUniqueId id;
        RCCL_OK(&c, ncclGetUniqueId(&id));
        ncclComm_t comm = nullptr;
        RCCL_OK(&c, ncclCommInitRank(&comm, 1, id, 0));
        D->comm = comm;
        const size_t nl = 1000, nr = 37;
        std::vector<char> hl(nl), hr(nr), gl(nr), gr(nl);
        for (size_t i = 0; i < nl; ++i) hl[i] = (char)(i * 7 + 1);
        for (size_t i = 0; i < nr; ++i) hr[i] = (char)(i * 5 + 2);
        char *sl, *sr, *rl, *rr;
        MPH_CK(ctx_dalloc(&c, &sl, nl)); MPH_CK(ctx_dalloc(&c, &sr, nr));
        MPH_CK(ctx_dalloc(&c, &rl, nr)); MPH_CK(ctx_dalloc(&c, &rr, nl));
        MPH_HIP_OK(&c, hipMemcpy(sl, hl.data(), nl, hipMemcpyHostToDevice));
        MPH_HIP_OK(&c, hipMemcpy(sr, hr.data(), nr, hipMemcpyHostToDevice));
        // left-going (sl) must arrive as from-right (rr); right-going (sr) as from-left (rl)
        MPH_CK(exchange(&c, c.stream, sl, nl, sr, nr, rl, nr, rr, nl));
        // a zero-byte direction is skipped on both sides
        MPH_CK(exchange(&c, c.stream, sl, 0, sr, nr, rl, nr, rr, 0));
        MPH_HIP_OK(&c, hipStreamSynchronize(c.stream));
        MPH_HIP_OK(&c, hipMemcpy(gl.data(), rl, nr, hipMemcpyDeviceToHost));
        MPH_HIP_OK(&c, hipMemcpy(gr.data(), rr, nl, hipMemcpyDeviceToHost));
        if (gl != hr || gr != hl) return ctx_fail(&c, MPH_ERR_RCCL, "RCCL self-exchange delivered wrong bytes");
        // the same exchange captured into a hipGraph and replayed (slab steps replay RCCL calls
        // from captured graphs)
        MPH_HIP_OK(&c, hipMemset(rl, 0, nr));
        MPH_HIP_OK(&c, hipMemset(rr, 0, nl));
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        MPH_HIP_OK(&c, hipStreamBeginCapture(c.stream, hipStreamCaptureModeThreadLocal));
        const int rc = exchange(&c, c.stream, sl, nl, sr, nr, rl, nr, rr, nl);
        const hipError_t e = hipStreamEndCapture(c.stream, &g);
        MPH_CK(rc);
        MPH_HIP_OK(&c, e);
        const hipError_t ei = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        MPH_HIP_OK(&c, ei);
        for (int rep = 0; rep < 2; ++rep) MPH_HIP_OK(&c, hipGraphLaunch(ge, c.stream));
        MPH_HIP_OK(&c, hipStreamSynchronize(c.stream));
        (void)hipGraphExecDestroy(ge);
        MPH_HIP_OK(&c, hipMemcpy(gl.data(), rl, nr, hipMemcpyDeviceToHost));
        MPH_HIP_OK(&c, hipMemcpy(gr.data(), rr, nl, hipMemcpyDeviceToHost));
        if (gl != hr || gr != hl) return ctx_fail(&c, MPH_ERR_RCCL, "graph-replayed RCCL exchange delivered wrong bytes");
        // the early send's pattern (dist_enqueue_step): per step the exchange forks onto a second
        // stream after an event of the main stream, main-stream work runs beside it, and the
        // next step joins it -- three chained steps in one captured graph, replayed twice
        hipStream_t s2 = nullptr;
        hipEvent_t es = nullptr, ex = nullptr;
        MPH_HIP_OK(&c, hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        MPH_HIP_OK(&c, hipEventCreateWithFlags(&es, hipEventDisableTiming));
        MPH_HIP_OK(&c, hipEventCreateWithFlags(&ex, hipEventDisableTiming));
        char* side;
        MPH_CK(ctx_dalloc(&c, &side, 1 << 20));
        MPH_HIP_OK(&c, hipMemset(rl, 0, nr));
        MPH_HIP_OK(&c, hipMemset(rr, 0, nl));
        MPH_HIP_OK(&c, hipStreamBeginCapture(c.stream, hipStreamCaptureModeThreadLocal));
        int rc2 = MPH_OK;
        for (int k = 0; k < 3 && rc2 == MPH_OK; ++k) {
            if (k > 0) (void)hipStreamWaitEvent(c.stream, ex, 0);
            (void)hipEventRecord(es, c.stream);
            (void)hipStreamWaitEvent(s2, es, 0);
            rc2 = exchange(&c, s2, sl, nl, sr, nr, rl, nr, rr, nl);
            (void)hipEventRecord(ex, s2);
            (void)hipMemsetAsync(side, k, 1 << 20, c.stream);   // work beside the exchange
        }
        (void)hipStreamWaitEvent(c.stream, ex, 0);
        const hipError_t e2 = hipStreamEndCapture(c.stream, &g);
        MPH_CK(rc2);
        MPH_HIP_OK(&c, e2);
        const hipError_t ei2 = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        MPH_HIP_OK(&c, ei2);
        for (int rep = 0; rep < 2; ++rep) MPH_HIP_OK(&c, hipGraphLaunch(ge, c.stream));
        MPH_HIP_OK(&c, hipStreamSynchronize(c.stream));
        (void)hipGraphExecDestroy(ge);
        (void)hipEventDestroy(es);
        (void)hipEventDestroy(ex);
        (void)hipStreamDestroy(s2);
        MPH_HIP_OK(&c, hipMemcpy(gl.data(), rl, nr, hipMemcpyDeviceToHost));
        MPH_HIP_OK(&c, hipMemcpy(gr.data(), rr, nl, hipMemcpyDeviceToHost));
        if (gl != hr || gr != hl)
            return ctx_fail(&c, MPH_ERR_RCCL, "forked graph-replayed RCCL exchanges delivered wrong bytes");
        return MPH_OK;
    };
    status = run();
    ctx_set_global_error(c.err);
    (void)hipStreamSynchronize(c.stream);
    dist_free(&c);
    for (void* p : c.allocs) (void)hipFree(p);
    if (c.stream) (void)hipStreamDestroy(c.stream);
    return status;
}

int mph_dist_overlap(const MphCtx* c, double* out5)
{
    if (!c || !out5) return MPH_ERR_ARG;
    for (int k = 0; k < 5; ++k) out5[k] = -1.0;
    if (!c->dist) return MPH_OK;
    const MphDist& D = *c->dist;
    out5[0] = D.overlap ? 1.0 : 0.0;
    out5[1] = D.overlap_mode;
    for (int k = 0; k < 3; ++k) out5[2 + k] = D.probe_ms[k];
    return MPH_OK;
}

int mph_dist_info(const MphCtx* c, int* out8)
{
    if (!c || !out8) return MPH_ERR_ARG;
    std::memset(out8, 0, 8 * sizeof(int));
    if (!c->dist) {
        out8[0] = 1;
        return MPH_OK;
    }
    const MphDist& D = *c->dist;
    // the RCCL communicator's own size (0 under the host-staged transport, which has none)
    int count = 0;
    if (D.rccl && D.comm && ncclCommCount((ncclComm_t)D.comm, &count) != ncclSuccess) count = -1;
    out8[0] = D.nranks;
    out8[1] = D.rank;
    out8[2] = count;
    out8[3] = D.graphs ? 1 : 0;
    out8[4] = D.cap;
    out8[5] = std::max(D.cap_sl, D.cap_sr);
    out8[6] = std::max(D.cap_rl, D.cap_rr);
    out8[7] = c->n;
    return MPH_OK;
}

int mph_owned_count(const MphCtx* c)
{
    if (!c) return -1;
    return c->dist ? c->dist->n_own : c->n_glob;
}

int mph_owned_ids(MphCtx* c, int* out)
{
    if (!c || !out) return MPH_ERR_ARG;
    if (!c->dist) {
        for (int i = 0; i < c->n_glob; ++i) out[i] = i;
        return MPH_OK;
    }
    MPH_HIP_OK(c, hipSetDevice(c->device));
    std::vector<int> id(c->n);
    MPH_HIP_OK(c, hipMemcpyAsync(id.data(), c->B.id, sizeof(int) * c->n, hipMemcpyDeviceToHost, c->stream));
    MPH_HIP_OK(c, hipStreamSynchronize(c->stream));
    int k = 0;
    for (int i = 0; i < c->n; ++i)
        if (id[i] >= 0) {
            if (k >= c->dist->n_own) return ctx_fail(c, MPH_ERR_CAPACITY, "owned id count mismatch");
            out[k++] = id[i];
        }
    std::sort(out, out + k);
    return k == c->dist->n_own ? MPH_OK : ctx_fail(c, MPH_ERR_CAPACITY, "owned id count mismatch");
}

int mph_slab_bounds(const MphConfig* cfg, int rank, int nranks, int axis, const double* cuts, double* out3)
{
    if (!cfg || !out3 || nranks < 1 || rank < 0 || rank >= nranks || axis < 0 || axis > 2) return MPH_ERR_ARG;
    HostDerived h{};
    derive_constants(*cfg, h);
    std::string err;
    if (check_cuts(h, axis, nranks, cuts, err) != MPH_OK) return MPH_ERR_ARG;
    DevParams P{};
    make_dev_params(*cfg, h, 0, 0, P);
    slab_of(h, axis, rank, nranks, cuts, out3[0], out3[1]);
    out3[2] = halo_width(P);
    return MPH_OK;
}

int mph_slab_window(const MphConfig* cfg, int rank, int nranks, int axis, const double* cuts, double* out2)
{
    double b[3];
    const int rc = mph_slab_bounds(cfg, rank, nranks, axis, cuts, b);
    if (rc != MPH_OK) return rc;
    if (!out2) return MPH_ERR_ARG;
    // two halo widths, each including the elastic particles' displacement margin, so that the
    // first redistribution's capacity estimate (dist_setup) and the structure lists of the owned
    // elastic particles (calculateInitialNeighbor reach) see every particle they need
    const double m = 2.0 * (b[2] + kStructMargin * cfg->particle_spacing);
    out2[0] = b[0] - m;
    out2[1] = b[1] + m;
    return MPH_OK;
}

int mph_slab_owner(const MphConfig* cfg, int nranks, int axis, const double* cuts, double x)
{
    if (!cfg || nranks < 1 || axis < 0 || axis > 2) return MPH_ERR_ARG;
    HostDerived h{};
    derive_constants(*cfg, h);
    std::string err;
    if (check_cuts(h, axis, nranks, cuts, err) != MPH_OK) return MPH_ERR_ARG;
    const double a = wrap_coord(h, axis, x);
    for (int r = 0; r < nranks; ++r) {
        double lo, hi;
        slab_of(h, axis, r, nranks, cuts, lo, hi);
        if (slab_owns(a, lo, hi, r == 0, r == nranks - 1)) return r;
    }
    return MPH_ERR_DOMAIN;
}

}  // extern "C"
