// mph_ctx.hip -- the C ABI of include/mph_gpu.h: device context, uploads, graph-replayed steps,
// field download in the reference's AoS layout and original particle order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "mph_ctx.h"

using namespace mph;

namespace mph {

int ctx_fail(MphCtx* c, int code, const std::string& msg)
{
    if (c) c->err = msg;
    return code;
}

int ctx_hip_fail(MphCtx* c, hipError_t e, const char* what)
{
    return ctx_fail(c, e == hipErrorOutOfMemory ? MPH_ERR_DEVICE_OOM : MPH_ERR_HIP,
                    std::string(what) + ": " + hipGetErrorString(e));
}

void* ctx_alloc(MphCtx* c, size_t bytes, int* status)
{
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) {
        *status = ctx_fail(c, e == hipErrorOutOfMemory ? MPH_ERR_DEVICE_OOM : MPH_ERR_HIP,
                           "hipMalloc(" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
        return nullptr;
    }
    c->allocs.push_back(q);
    *status = MPH_OK;
    return q;
}

// Error flags raised by the kernels (DevState.overflow bits).
int ctx_state_status(MphCtx* c, const DevState& hs)
{
    if (hs.overflow & 4)
        return ctx_fail(c, MPH_ERR_NONFINITE, "non-finite particle position (diverged state)");
    if (hs.overflow & 1)
        return ctx_fail(c, MPH_ERR_NEIGHBOR_OVERFLOW, "a particle has more than 512 neighbours");
    if (hs.overflow & 2) return ctx_fail(c, MPH_ERR_CAPACITY, "a particle moved past a neighbouring slab");
    if (hs.overflow & 64)   // k_place: a cell start + slot past the particle count (never a fault)
        return ctx_fail(c, MPH_ERR_HIP, "cell sort: histogram inconsistent with the keys (placement out of range)");
    return MPH_OK;
}

void ctx_fill_launch(MphCtx* c)
{
    Launch& L = c->L;
    set_uniforms(c->P);
    // MPH_LIST_FULL=1: the lists keep every neighbour within the search radius, like the reference's
    // Neighbor[] (mph_neighbor_rows needs them); else only those the passes' sums can take
    if (std::getenv("MPH_LIST_FULL") && std::atoi(std::getenv("MPH_LIST_FULL")) == 1) c->P.rlf = 3.0e38f;
    L.P = &c->P;
    L.T = c->dT;
    L.st = c->dst;
    L.stream = c->stream;
    L.prof = nullptr;
    // rank_of (original id -> sorted index) has no reader on the single-GPU path (fields are
    // returned through A.id), so k_rank_scatter skips that scatter; slab mode uses dst_of.
    L.A = c->A; L.B = c->B; L.rank_of = nullptr; L.dst_of = nullptr;
    L.key = c->key; L.slot = c->slot; L.tmp = c->tmp; L.cnt = c->cnt; L.start = c->start; L.bsum = c->bsum;
    L.nbr = c->nbr; L.ncount = c->ncount; L.nbcount = c->nbcount; L.lhdr = c->lhdr; L.lgap = c->lgap;
    // work-balanced XCD map of the passes from this many particles (MPH_XCD_BAL_MIN: tests force it
    // on small cases, the default keeps it off below 2^20 where the split kernel costs more)
    const char* bm = std::getenv("MPH_XCD_BAL_MIN");
    L.xcd_bal_min = bm && *bm ? std::atoi(bm) : (1 << 20);
    L.pres = c->pres; L.gx = c->gx; L.gy = c->gy; L.gz = c->gz; L.pa = c->pa;
    L.force = c->force; L.acc = c->acc; L.fpart = c->fpart; L.rec = c->rec;
    L.dens_a = c->dens_a; L.vstrain = c->vstrain; L.divp = c->divp;
    L.S = &c->Sd;
}

// calculateVirialStressAtParticle evaluates the step's lists at the positions after the step
// (main.cpp:672-673, 3077-3318): a pair of the shell MaxRadius < r <= MaxRadius + MARGIN at the search
// may have moved inside a radius by then, so the virial needs the reference's whole lists.  With
// the lists kept to the passes' radius (DevParams.rlf) the step's search is repeated over the same
// sorted set A and cell table (unchanged since the step's sort) storing every neighbour -- the
// lists the step would have built with MPH_LIST_FULL=1; the XCD work histogram is left alone.
int virial_full_lists(MphCtx* c)
{
    if (c->P.rlf >= 3.0e38f) return MPH_OK;
    DevParams Pf = c->P;
    Pf.rlf = 3.0e38f;
    Launch L = c->L;
    L.P = &Pf;
    L.xcd_bal_min = 0x7fffffff;
    launch_neighbors(L);
    MPH_HIP_OK(c, hipGetLastError());
    return MPH_OK;
}
}  // namespace mph

namespace {

int fail(MphCtx* c, int code, const std::string& msg) { return ctx_fail(c, code, msg); }

#define HIP_OK(ctx, expr) MPH_HIP_OK(ctx, expr)
#define CK(expr) MPH_CK(expr)

template <typename T>
int dalloc(MphCtx* c, T** p, size_t count)
{
    return ctx_dalloc(c, p, count);
}

void fill_launch(MphCtx* c) { ctx_fill_launch(c); }

// Force and Acceleration (main.cpp:2085-2096, 2892-2956) are outputs only: no kernel reads them,
// and every step overwrites all of them.  So only the last step of a replayed batch stores them
// (pass B -6 % at D1M); mph_get after any mph_step sees the last step's values as before.  The
// same holds in pass A for DensityA, VolStrainP, DivergenceP and, without surface tension (pass B
// then reads neither), GravityCenter and PressureA.  The virial (k_virial) runs after a batch.
// ev (phase timing, else null): three events recorded on the stream at the step's phase
// boundaries -- before the sort, after the search (neighbour search = sort + search, as the
// reference's calculateNeighbor holds its own cell sort), after the elastic substeps.
void enqueue_step(const Launch& L, bool last, hipEvent_t* ev = nullptr)
{
    if (ev) (void)hipEventRecord(ev[0], L.stream);
    launch_sort(L, 1);
    Launch La = L;
    if (!last) {
        La.dens_a = La.vstrain = La.divp = nullptr;
        if (!L.P->surface) La.gx = La.gy = La.gz = La.pa = nullptr;
    }
    if (ev) {   // phase timing: the boundary between the search and pass A
        launch_neighbors(La);
        (void)hipEventRecord(ev[1], L.stream);
        launch_pass_a(La);
    } else {
        launch_search_pass_a(La);
    }
    if (last) {
        launch_pass_b(L);
    } else {
        Launch Lb = L;
        Lb.force = nullptr;
        Lb.acc = nullptr;
        launch_pass_b(Lb);
    }
    launch_structure(L, last);
    if (ev) (void)hipEventRecord(ev[2], L.stream);
}

// store_last = false: no step of the graph stores the output-only fields (graph1t, the steps of a
// remainder before its last one)
int capture(MphCtx* c, int steps, hipGraphExec_t* out, bool store_last = true)
{
    hipGraph_t g = nullptr;
    HIP_OK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < steps; ++k) enqueue_step(c->L, store_last && k == steps - 1);
    HIP_OK(c, hipStreamEndCapture(c->stream, &g));
    HIP_OK(c, hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    HIP_OK(c, hipGraphDestroy(g));
    HIP_OK(c, hipGraphUpload(*out, c->stream));   // so the first launch costs what later ones do
    return MPH_OK;
}

// The step graphs, captured at the first mph_step whatever its count: a caller that warms up with
// fewer than 8 steps (the driver's bench: 5) would otherwise capture and upload the 8-step graph
// inside its first long run.
static int capture_graphs(MphCtx* c)
{
    if (!c->graph1) CK(capture(c, 1, &c->graph1));
    if (!c->graph1t) CK(capture(c, 1, &c->graph1t, false));
    if (!c->graph8) CK(capture(c, 8, &c->graph8));
    return MPH_OK;
}

// `left` (< 8) single steps: the output-only stores on the last one only, as in an 8-step batch
static int launch_singles(MphCtx* c, int left)
{
    for (; left > 1; --left) HIP_OK(c, hipGraphLaunch(c->graph1t, c->stream));
    if (left == 1) HIP_OK(c, hipGraphLaunch(c->graph1, c->stream));
    return MPH_OK;
}

// phase timing: the events of a batch of `steps` steps (three per step) into the neighbour /
// explicit sums
int accumulate_phases(MphCtx* c, const std::vector<hipEvent_t>& ev, int steps)
{
    HIP_OK(c, hipEventSynchronize(ev[3 * (size_t)steps - 1]));
    for (size_t k = 0; k + 2 < 3 * (size_t)steps; k += 3) {
        float a = 0.0f, b = 0.0f;
        HIP_OK(c, hipEventElapsedTime(&a, ev[k], ev[k + 1]));
        HIP_OK(c, hipEventElapsedTime(&b, ev[k + 1], ev[k + 2]));
        c->phase_ms[0] += a;
        c->phase_ms[1] += b;
    }
    return MPH_OK;
}

// Device sorted arrays -> host original order via the id arrays.
int download_vec(MphCtx* c, const double4* d, const int* ids, double* out, int width)
{
    const int n = c->n;
    std::vector<double4> h(n);
    std::vector<int> id(n);
    HIP_OK(c, hipMemcpyAsync(h.data(), d, sizeof(double4) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipMemcpyAsync(id.data(), ids, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; ++i) {
        if (id[i] < 0) continue;   // slab mode: ghost
        double* o = out + (size_t)width * id[i];
        o[0] = h[i].x;
        if (width > 1) { o[1] = h[i].y; o[2] = h[i].z; }
    }
    return MPH_OK;
}

template <typename T>
int download_scalar(MphCtx* c, const T* d, const int* ids, T* out)
{
    const int n = c->n;
    std::vector<T> h(n);
    std::vector<int> id(n);
    HIP_OK(c, hipMemcpyAsync(h.data(), d, sizeof(T) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipMemcpyAsync(id.data(), ids, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; ++i)
        if (id[i] >= 0) out[id[i]] = h[i];
    return MPH_OK;
}

// three SoA component arrays -> AoS double[n][3] in original order
int download_soa3(MphCtx* c, const double* dx, const double* dy, const double* dz, const int* ids,
                  double* out)
{
    const int n = c->n;
    std::vector<double> h(3 * (size_t)n);
    std::vector<int> id(n);
    const double* src[3] = {dx, dy, dz};
    for (int k = 0; k < 3; ++k)
        HIP_OK(c, hipMemcpyAsync(h.data() + (size_t)k * n, src[k], sizeof(double) * n, hipMemcpyDeviceToHost,
                                 c->stream));
    HIP_OK(c, hipMemcpyAsync(id.data(), ids, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; ++i)
        if (id[i] >= 0)
            for (int k = 0; k < 3; ++k) out[3 * (size_t)id[i] + k] = h[(size_t)k * n + i];
    return MPH_OK;
}

int download_w(MphCtx* c, const double4* d, const int* ids, double* out)
{
    const int n = c->n;
    std::vector<double4> h(n);
    std::vector<int> id(n);
    HIP_OK(c, hipMemcpyAsync(h.data(), d, sizeof(double4) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipMemcpyAsync(id.data(), ids, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; ++i)
        if (id[i] >= 0) out[id[i]] = h[i].w;
    return MPH_OK;
}

int download_struct_m33(MphCtx* c, const double* d, double* out)
{
    const int ns = c->Sd.n_own;   // slots computed here (slab mode: owned)
    std::memset(out, 0, sizeof(double) * 9 * (size_t)c->n_glob);
    if (ns == 0) return MPH_OK;
    const size_t fes = (size_t)c->Sd.fes;   // nine element planes (StructDev)
    std::vector<double> h(fes * 9);
    HIP_OK(c, hipMemcpyAsync(h.data(), d, sizeof(double) * 9 * fes, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    for (int s = 0; s < ns; ++s) {
        double* o = out + (size_t)9 * c->sl_orig[s];
        for (int e = 0; e < 9; ++e) o[e] = h[e * fes + s];
    }
    return MPH_OK;
}

// A launch's start event behind a cross-stream wait reads as early as the wait packet itself (the
// time the stream went idle), so each launch that follows a join also keeps a floor: an event on
// the other stream at the joined point; its start is the later of the two.
struct EventProfiler final : Profiler {
    struct Rec { std::string name; hipEvent_t a, b; int floor; };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> floors;
    std::map<hipStream_t, int> pending;
    bool events(const char* name, hipStream_t s, hipEvent_t* start, hipEvent_t* stop) override
    {
        Rec r{name, nullptr, nullptr, -1};
        const auto it = pending.find(s);
        if (it != pending.end()) {
            r.floor = it->second;
            pending.erase(it);
        }
        (void)hipEventCreate(&r.a);
        (void)hipEventCreate(&r.b);
        recs.push_back(r);
        *start = r.a;
        *stop = r.b;
        return true;
    }
    void join(hipStream_t waiting, hipStream_t from) override
    {
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        (void)hipEventRecord(e, from);
        floors.push_back(e);
        pending[waiting] = (int)floors.size() - 1;
    }
    ~EventProfiler() override
    {
        for (auto& r : recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
        for (auto e : floors) (void)hipEventDestroy(e);
    }
};

}  // namespace

extern "C" {

}  // extern "C"

namespace mph {

// Shared body of mph_create (dist == nullptr) and the slab-mode constructors of mph_dist.hip
// (dist != nullptr: only this rank's particles are uploaded, the cell grid covers its window).
static thread_local std::string g_create_error;   // mph_last_error(NULL) after a failed create

static int ctx_init(MphCtx* c, const MphConfig* cfg, int n, const int* property, const double* pos,
                    const double* pos0, const double* vel, int device, const int* ids, int n_glob)
{
    if (cfg->dim != 2 && cfg->dim != 3) return MPH_ERR_ARG;
    if (cfg->module < 0 || cfg->module > MPH_MODULE_NONE) return MPH_ERR_ARG;
    if (!(cfg->particle_spacing > 0.0) || !(cfg->dt > 0.0) || !(cfg->elastic_dt > 0.0)) return MPH_ERR_ARG;
    for (int i = 0; i < n; ++i)
        if (property[i] < 0 || property[i] >= kTypes) return MPH_ERR_ARG;
    c->cfg = *cfg;
    c->n = n;
    c->n_glob = n;
    if (ids) {
        if (!c->dist || n_glob < n) return MPH_ERR_ARG;
        for (int i = 0; i < n; ++i)
            if (ids[i] < 0 || ids[i] >= n_glob || (i > 0 && ids[i] <= ids[i - 1]))
                return fail(c, MPH_ERR_ARG, "slab-local creation: ids must be ascending original indices below n_glob");
        c->gid.assign(ids, ids + n);
        c->n_glob = n_glob;
    }
    c->device = device;
    c->time = cfg->time;
    HIP_OK(c, hipSetDevice(device));
    HIP_OK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    derive_constants(c->cfg, c->h);
    c->prop.assign(property, property + n);
    c->pos0.assign(pos0, pos0 + 3 * (size_t)n);
    std::string err;
    // the fixed Lagrangian structure lists: on the device for a single context (calculate-
    // InitialNeighbor + calculateNormalizer as kernels, launch_struct_init); in slab mode on the
    // host over the particles this rank was given, which also routes the static ghost slots
    // (dist_struct_setup).  MPH_STRUCT_INIT=host selects the host build everywhere.
    const char* sie = std::getenv("MPH_STRUCT_INIT");
    const bool gpu_init = !c->dist && !(sie && std::string(sie) == "host");
    CK(fail(c, build_structure(c->cfg, c->h, n, property, pos0, c->S, err, !gpu_init), err));
    const int ns = (int)c->S.orig.size();
    make_dev_params(c->cfg, c->h, n, ns, c->P);
    const double rc = std::sqrt(c->P.rc2);
    {
        // z slabs of a 3-D problem: z in the middle of the cell order, so the ghosts beyond both
        // faces are long runs (whole wavefronts) at the ends of every plane (DevParams.perm;
        // MPH_SLAB_PERM=0 keeps (x, y, z); =1..4 force an order on any 3-D context, =force
        // orders a single 3-D context the z-slab way -- A/B timing and the parity tests)
        const char* pe = std::getenv("MPH_SLAB_PERM");
        const std::string pv = pe ? pe : "";
        const bool zslab = cfg->dim == 3 && c->dist && c->dist->g.axis == 2;
        const bool forced = pv.size() == 1 && pv[0] >= '1' && pv[0] <= '4';
        c->P.perm = 0;
        if (cfg->dim == 3 && (forced || pv == "force" || (zslab && pv != "0")))
            c->P.perm = forced ? pv[0] - '0' : choose_cell_order(c->h, n, pos, rc);
        int r = choose_grid(c->h, cfg->dim, rc, kContigReach, c->P.gc, c->P.ginv, err, c->P.perm);
        if (r != MPH_OK) return fail(c, r, err);
        set_uniforms(c->P);
    }
    // interior box for the wave-uniform fast minimum image (k_neighbors / passes): >= 3 cells
    // (+1e-9 relative margin) from every periodic face; needs > 12 cells on every active axis
    // (stencil half-width + 1 cells from every periodic face; the candidate offsets then stay
    // below a quarter of the domain width, which needs > 4 x that many cells on every axis)
    c->P.sa = kContigReach;
    c->P.fast_ok = 1;
    c->P.seam_always = 0;
    // the grid's origin in an empty band of the initial particles (choose_grid_origin;
    // MPH_GRID_SHIFT=0 keeps dmin): the search's interior box is then in grid offsets
    const char* gsh = std::getenv("MPH_GRID_SHIFT");
    const bool shift = !(gsh && gsh[0] == '0');
    for (int d = 0; d < 3; ++d) {
        if (d == 2 && cfg->dim == 2) {
            c->P.inner_lo[d] = c->P.sinner_lo[d] = -1e300;
            c->P.inner_hi[d] = c->P.sinner_hi[d] = 1e300;
            continue;
        }
        const int m = stencil_margin(c->P, d);
        if (c->P.gc[d] <= 4 * m) c->P.fast_ok = 0;
        const double cw = c->h.dw[d] / c->P.gc[d];
        c->P.inner_lo[d] = c->h.dmin[d] + m * cw * (1.0 + 1e-9);
        c->P.inner_hi[d] = c->h.dmax[d] - m * cw * (1.0 + 1e-9);
        const int s0 = shift && c->P.fast_ok ? choose_grid_origin(c->h, n, pos, d, c->P.gc[d], m) : 0;
        c->P.corg[d] = c->h.dmin[d] + s0 * cw;
        c->P.sinner_lo[d] = m * cw * (1.0 + 1e-9);
        c->P.sinner_hi[d] = c->h.dw[d] - m * cw * (1.0 + 1e-9);
    }
    // slab mode: owned subset, local window grid along the slab axis, array capacity
    std::vector<int> owned;
    int cap = n;
    if (c->dist) {
        CK(dist_setup(c, pos, owned));
        cap = c->dist->cap;
        c->n = (int)owned.size();
        c->P.n = c->n;
    }
    if (cap > kIndexMask)
        return fail(c, MPH_ERR_UNSUPPORTED, "more than 2^28 particles in one context (neighbour-list entries "
                                            "carry the type in their top bits)");
    if ((long long)cap * 48 >= (long long)kGatherOob)
        return fail(c, MPH_ERR_UNSUPPORTED, "more than 89 million particles in one context (the list passes "
                                            "gather with 32-bit byte offsets)");
    {
        // the search addresses the cell table with 32-bit byte offsets (buffer descriptors)
        const long long nc = (long long)c->P.gc[0] * c->P.gc[1] * c->P.gc[2];
        if (nc + 1 > (1LL << 30))
            return fail(c, MPH_ERR_UNSUPPORTED, "cell grid of " + std::to_string(nc) +
                                                    " cells: more than 2^30 (4 GiB of cell starts)");
        c->P.ncell = (int)nc;
    }
    // tables
    for (int t = 0; t < kTypes; ++t) {
        for (int u = 0; u < kTypes; ++u) {
            c->T.ratio[t * kTypes + u] = c->P.ratio[t][u];
            c->T.mu_ij[t * kTypes + u] = c->P.mu_ij[t][u];
        }
        c->T.cofa[t] = c->P.cofa[t];
        c->T.mass[t] = c->P.mass[t];
        c->T.inv_mass[t] = c->P.inv_mass[t];
        c->T.bulk[t] = c->P.bulk[t];
        c->T.bulk_visc[t] = c->P.bulk_visc[t];
    }
    // device allocations (capacity `cap` per particle array)
    const size_t ntile = ((size_t)cap + kTile - 1) / kTile;
    CK(dalloc(c, &c->dT, 1));
    CK(dalloc(c, &c->dst, 1));
    for (Soa* s : {&c->A, &c->B}) {
        const size_t m = (size_t)cap + kPad;
        CK(dalloc(c, &s->x, m)); CK(dalloc(c, &s->y, m)); CK(dalloc(c, &s->z, m));
        CK(dalloc(c, &s->vx, m)); CK(dalloc(c, &s->vy, m)); CK(dalloc(c, &s->vz, m));
        CK(dalloc(c, &s->type, m)); CK(dalloc(c, &s->id, m));
    }
    CK(dalloc(c, &c->A.p6, 3 * (size_t)cap));
    // the search's FP32 candidate records (kPad past the last)
    CK(dalloc(c, &c->A.f4, (size_t)cap + kPad));
    CK(dalloc(c, &c->rank_of, cap));
    CK(dalloc(c, &c->key, cap)); CK(dalloc(c, &c->slot, cap)); CK(dalloc(c, &c->tmp, cap));
    CK(dalloc(c, &c->cnt, c->P.ncell)); CK(dalloc(c, &c->start, (size_t)c->P.ncell + 1));
    // the cell scan's block totals (k_scan_reduce; structure init)
    const size_t bs = (size_t)c->P.ncell / 4096 + 2;   // bsum_stride (mph_kernels.hip)
    CK(dalloc(c, &c->bsum, bs));
    CK(dalloc(c, &c->nbr, ntile * kTileStride)); CK(dalloc(c, &c->ncount, cap));
    CK(dalloc(c, &c->nbcount, cap));
    // the lists' row jumps: a header word per wave, a word of gap starts per lane (whole tiles)
    CK(dalloc(c, &c->lhdr, ntile)); CK(dalloc(c, &c->lgap, ntile * kTile));
    CK(dalloc(c, &c->pres, cap)); CK(dalloc(c, &c->gx, cap)); CK(dalloc(c, &c->gy, cap)); CK(dalloc(c, &c->gz, cap));
    CK(dalloc(c, &c->pa, cap)); CK(dalloc(c, &c->force, cap)); CK(dalloc(c, &c->acc, cap));
    CK(dalloc(c, &c->fpart, cap)); CK(dalloc(c, &c->rec, cap));
    CK(dalloc(c, &c->dens_a, cap)); CK(dalloc(c, &c->vstrain, cap)); CK(dalloc(c, &c->divp, cap));
    HIP_OK(c, hipMemsetAsync(c->cnt, 0, sizeof(int) * c->P.ncell, c->stream));
    HIP_OK(c, hipMemsetAsync(c->bsum, 0, sizeof(int) * bs, c->stream));
    HIP_OK(c, hipMemsetAsync(c->force, 0, sizeof(double4) * std::max(cap, 1), c->stream));
    HIP_OK(c, hipMemsetAsync(c->acc, 0, sizeof(double4) * std::max(cap, 1), c->stream));
    HIP_OK(c, hipMemcpyAsync(c->dT, &c->T, sizeof(DevTables), hipMemcpyHostToDevice, c->stream));
    DevState st{};
    st.time = cfg->time;
    for (int t = 0; t < kTypes; ++t)
        for (int d = 0; d < 3; ++d) {
            st.wall_c[t][d] = cfg->wall_center[t][d];
            st.wall_vel[t][d] = cfg->wall_velocity[t][d];
            st.wall_omega[t][d] = cfg->wall_omega[t][d];
            for (int e = 0; e < 3; ++e) st.wall_rot[t][d][e] = c->h.wall_rot[t][d][e];
        }
    HIP_OK(c, hipMemcpyAsync(c->dst, &st, sizeof(DevState), hipMemcpyHostToDevice, c->stream));
    {
        // upload into the B set (original order, id = file index); the init sort reorders it
        const int m = c->n;
        std::vector<int> sel(m);
        for (int i = 0; i < m; ++i) sel[i] = c->dist ? owned[i] : i;
        std::vector<double> comp(m);
        std::vector<int> gids(m), types(m);
        double* dstc[6] = {c->B.x, c->B.y, c->B.z, c->B.vx, c->B.vy, c->B.vz};
        for (int k = 0; k < 6; ++k) {
            const double* src = k < 3 ? pos : vel;
            for (int i = 0; i < m; ++i) comp[i] = src[3 * (size_t)sel[i] + (k % 3)];
            HIP_OK(c, hipMemcpy(dstc[k], comp.data(), sizeof(double) * m, hipMemcpyHostToDevice));
        }
        for (int i = 0; i < m; ++i) { gids[i] = glob_id(c, sel[i]); types[i] = property[sel[i]]; }
        HIP_OK(c, hipMemcpy(c->B.type, types.data(), sizeof(int) * m, hipMemcpyHostToDevice));
        HIP_OK(c, hipMemcpy(c->B.id, gids.data(), sizeof(int) * m, hipMemcpyHostToDevice));
    }
    // elastic solid: local slots = [computed here | ghosts] (single GPU: every slot, no ghosts)
    if (ns > 0) {
        StructDev& D = c->Sd;
        StructureInit& S = c->S;
        std::vector<int> lsl;   // local slot -> global slot
        int no = ns, ni = ns;
        if (c->dist) {
            CK(dist_struct_setup(c, lsl, no, ni));
        } else {
            lsl.resize(ns);
            for (int s = 0; s < ns; ++s) lsl[s] = s;
        }
        const int nl = (int)lsl.size();
        std::vector<int> loc(ns, -1);
        for (int k = 0; k < nl; ++k) loc[lsl[k]] = k;
        D.n_own = no;
        D.n_inner = ni;
        c->sl_orig.resize(nl);
        for (int k = 0; k < nl; ++k) c->sl_orig[k] = glob_id(c, S.orig[lsl[k]]);
        c->sl_s.assign(lsl.begin(), lsl.begin() + no);
        const int sd = c->P.dim;
        CK(dalloc(c, &D.orig, nl)); CK(dalloc(c, &D.ocnt, std::max(no, 1))); CK(dalloc(c, &D.icnt, std::max(no, 1)));
        CK(dalloc(c, &D.bidx, nl));
        CK(dalloc(c, &D.wx0, nl));
        CK(dalloc(c, &D.L, (size_t)nl * 9)); CK(dalloc(c, &D.lame, nl)); CK(dalloc(c, &D.inv_rho, nl));
        CK(dalloc(c, &D.clamp, nl)); CK(dalloc(c, &D.x0, nl)); CK(dalloc(c, &D.x, nl)); CK(dalloc(c, &D.v, nl));
        CK(dalloc(c, &D.u, nl)); CK(dalloc(c, &D.P, (size_t)nl * (sd == 2 ? 1 : 3))); CK(dalloc(c, &D.F, (size_t)nl * 9));
        CK(dalloc(c, &D.E, (size_t)nl * 9)); CK(dalloc(c, &D.S, (size_t)nl * 9));
        D.fes = nl;
        std::vector<double2> lame(nl);
        std::vector<double> irho(nl);
        std::vector<int> clamp(nl);
        std::vector<double4> x0(nl);
        for (int s = 0; s < nl; ++s) {
            const int g = lsl[s];
            const int i = S.orig[g];
            const int t = property[i];
            lame[s] = make_double2(S.lame_l[g], S.lame_m[g]);
            irho[s] = 1.0 / cfg->density[t];
            const double* p0 = pos0 + 3 * (size_t)i;
            int cl = 0;   // updateElasticPosition module clamps (main.cpp:1918-2044)
            switch (cfg->module) {
            case MPH_MODULE_BAR: cl = p0[0] < 0.001 ? 1 : 0; break;
            case MPH_MODULE_DAM: cl = p0[1] < 0.002 ? 1 : 0; break;
            case MPH_MODULE_TUREK_HRON: cl = p0[0] < 0.205 ? 2 : 0; break;
            case MPH_MODULE_ROLLING1: cl = p0[1] < 0.003 ? 1 : 0; break;
            case MPH_MODULE_HYDROELASTIC: cl = (p0[0] < 0.01 || p0[0] > 1.99) ? 1 : 0; break;
            default: cl = 0;
            }
            clamp[s] = cl;
            x0[s] = make_double4(p0[0], p0[1], p0[2], (double)t);
        }
        auto up = [&](auto* d, const auto& v) {
            return hipMemcpyAsync(d, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice, c->stream);
        };
        HIP_OK(c, up(D.x0, x0));
        if (gpu_init) {
            // calculateInitialNeighbor + calculateNormalizer on the device (single context: the
            // local slots are all slots, in file order); the host keeps counts and normalizers
            // for mph_get
            fill_launch(c);
            auto alloc = [](void* ctx, size_t bytes) -> void* {
                int st = MPH_OK;
                return ctx_alloc((MphCtx*)ctx, bytes, &st);
            };
            const int r = launch_struct_init(c->L, ns, D.x0, c->key, c->slot, c->tmp, c->rank_of, D.ocnt, D.icnt,
                                             &D.eo_nb, &D.wo, &D.ei_nb, &D.wi, D.L, D.wx0, alloc, c);
            if (r == -2) return fail(c, MPH_ERR_NEIGHBOR_OVERFLOW, "a structure particle has >= 512 initial neighbours");
            if (r == -3) return fail(c, MPH_ERR_DEVICE_OOM, "structure list allocation failed");
            if (r != 0) return fail(c, MPH_ERR_HIP, "structure initialisation kernels failed");
            S.count.resize(ns);
            S.normalizer.resize((size_t)ns * 9);
            HIP_OK(c, hipMemcpyAsync(S.count.data(), D.ocnt, sizeof(int) * ns, hipMemcpyDeviceToHost, c->stream));
            HIP_OK(c, hipMemcpyAsync(S.normalizer.data(), D.L, sizeof(double) * 9 * ns, hipMemcpyDeviceToHost,
                                     c->stream));
            HIP_OK(c, hipStreamSynchronize(c->stream));
        } else {
            // ELL tiles of the host-built fixed out-list and of its transpose (StructDev), computed slots only
            const size_t ntile_s = ((size_t)std::max(no, 1) + 63) / 64;
            std::vector<int> ocnt(std::max(no, 1), 0), icnt(std::max(no, 1), 0);
            int wo = 0, wi = 0;
            for (int s = 0; s < no; ++s) {
                const int g = lsl[s];
                ocnt[s] = S.offset[g + 1] - S.offset[g];
                icnt[s] = S.in_offset[g + 1] - S.in_offset[g];
                wo = std::max(wo, ocnt[s]);
                wi = std::max(wi, icnt[s]);
            }
            wo = std::max(wo, 1);
            wi = std::max(wi, 1);
            D.wo = wo;
            D.wi = wi;
            std::vector<int> eo_nb(ntile_s * wo * 64, 0), ei_nb(ntile_s * wi * 64, 0);
            std::vector<double4> wx0(nl, make_double4(0.0, 0.0, 0.0, 0.0));
            for (int s = 0; s < no; ++s) {
                const int g = lsl[s];
                const size_t base_o = (size_t)(s >> 6) * wo * 64 + (s & 63);
                double c3[3] = {0.0, 0.0, 0.0};
                for (int k = 0; k < ocnt[s]; ++k) {
                    const size_t q = S.offset[g] + k;
                    const double* pr = &S.pair_out[4 * q];
                    eo_nb[base_o + (size_t)k * 64] = loc[S.nbr[q]];
                    for (int d = 0; d < 3; ++d) c3[d] += pr[3] * pr[d];
                }
                wx0[s] = make_double4(c3[0], c3[1], c3[2], 0.0);
                const size_t base_i = (size_t)(s >> 6) * wi * 64 + (s & 63);
                for (int k = 0; k < icnt[s]; ++k) {
                    const size_t q = S.in_offset[g] + k;
                    ei_nb[base_i + (size_t)k * 64] = loc[S.in_nbr[q]];
                }
            }
            for (int e : eo_nb) if (e < 0) return fail(c, MPH_ERR_DOMAIN, "structure list leaves the ghost slots");
            for (int e : ei_nb) if (e < 0) return fail(c, MPH_ERR_DOMAIN, "structure list leaves the ghost slots");
            std::vector<double> Lm((size_t)nl * 9);
            for (int s = 0; s < nl; ++s)
                std::memcpy(&Lm[(size_t)9 * s], &S.normalizer[(size_t)9 * lsl[s]], sizeof(double) * 9);
            CK(dalloc(c, &D.eo_nb, eo_nb.size()));
            CK(dalloc(c, &D.ei_nb, ei_nb.size()));
            HIP_OK(c, up(D.ocnt, ocnt)); HIP_OK(c, up(D.icnt, icnt));
            HIP_OK(c, up(D.eo_nb, eo_nb));
            HIP_OK(c, up(D.ei_nb, ei_nb));
            HIP_OK(c, up(D.wx0, wx0));
            HIP_OK(c, up(D.L, Lm));
        }
        HIP_OK(c, hipMemcpyAsync(D.orig, c->sl_orig.data(), sizeof(int) * nl, hipMemcpyHostToDevice, c->stream));
        {
            std::vector<int> slot_of((size_t)c->n_glob, -1);
            for (int s = 0; s < no; ++s) slot_of[c->sl_orig[s]] = s;
            CK(dalloc(c, &D.slot_of, slot_of.size()));
            HIP_OK(c, hipMemcpy(D.slot_of, slot_of.data(), sizeof(int) * slot_of.size(), hipMemcpyHostToDevice));
        }
        HIP_OK(c, up(D.lame, lame));
        HIP_OK(c, up(D.inv_rho, irho));
        HIP_OK(c, up(D.clamp, clamp));
        HIP_OK(c, hipMemsetAsync(D.P, 0, sizeof(double4) * (sd == 2 ? 1 : 3) * nl, c->stream));
        HIP_OK(c, hipMemsetAsync(D.u, 0, sizeof(double4) * nl, c->stream));
        HIP_OK(c, hipMemsetAsync(D.bidx, 0, sizeof(int) * nl, c->stream));
        for (double* m : {D.F, D.E, D.S})
            HIP_OK(c, hipMemsetAsync(m, 0, sizeof(double) * 9 * nl, c->stream));
        HIP_OK(c, hipStreamSynchronize(c->stream));
    }
    fill_launch(c);
    if (c->dist) {
        // slab mode: allocations of the exchange, then the initial ghost exchange + init sums
        CK(dist_alloc(c));
        CK(dist_init(c));
    } else {
        // initialisation sums, main.cpp:565-568 (calculateNeighbor, DensityA, GravityCenter, DensityP)
        launch_sort(c->L, 0);
        launch_search_pass_a(c->L);
    }
    HIP_OK(c, hipGetLastError());
    HIP_OK(c, hipStreamSynchronize(c->stream));
    {
        DevState hs;
        HIP_OK(c, hipMemcpy(&hs, c->dst, kStateHead, hipMemcpyDeviceToHost));
        CK(ctx_state_status(c, hs));
    }
    return MPH_OK;
}

void ctx_set_global_error(const std::string& msg) { g_create_error = msg; }

int ctx_create(MphCtx** out, const MphConfig* cfg, int n, const int* property, const double* pos,
               const double* pos0, const double* vel, int device, MphDist* dist, const int* ids, int n_glob)
{
    g_create_error.clear();
    if (!out || !cfg || n < 0 || (n > 0 && (!property || !pos || !pos0 || !vel))) {
        delete dist;
        g_create_error = "invalid argument";
        return MPH_ERR_ARG;
    }
    *out = nullptr;
    MphCtx* c = new MphCtx();
    c->dist = dist;
    const int r = ctx_init(c, cfg, n, property, pos, pos0, vel, device, ids, n_glob);
    if (r != MPH_OK) {
        g_create_error = c->err.empty() ? "mph_create failed with status " + std::to_string(r) : c->err;
        mph_destroy(c);
        return r;
    }
    *out = c;
    return MPH_OK;
}

}  // namespace mph

extern "C" {

int mph_create(MphCtx** out, const MphConfig* cfg, int n, const int* property, const double* pos,
               const double* pos0, const double* vel, int device)
{
    return ctx_create(out, cfg, n, property, pos, pos0, vel, device, nullptr);
}

// Step batching: launch the steps accepted but not launched (single-step graphs, each storing the
// output-only fields, so the last one leaves them current) and read the error flags of everything
// launched.  Every entry point that reads or changes the state, or waits for it, calls this first.
static int ctx_flush(MphCtx* c)
{
    if (!c->pending && !c->unchecked) return MPH_OK;
    HIP_OK(c, hipSetDevice(c->device));
    if (c->pending) CK(capture_graphs(c));
    if (c->pending) CK(launch_singles(c, c->pending));
    c->pending = 0;
    c->unchecked = false;
    DevState hs;
    HIP_OK(c, hipMemcpyAsync(&hs, c->dst, kStateHead, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    return ctx_state_status(c, hs);
}

// mph_step with batching on: the steps are counted and launched 8 at a time from the 8-step graph
// (output-only fields stored on each batch's last step, as a multi-step mph_step does); the error
// flags of the last launched batch are copied back behind it and read without waiting once they
// have landed, so an error surfaces at most a batch or two late, and at the latest at the next
// flush point (mph_synchronize, mph_get, the writers, ...).
static int step_batched(MphCtx* c, int nsteps)
{
    for (int k = 0; k < nsteps; ++k) c->time += c->cfg.dt;
    c->stepped = true;
    c->pending += nsteps;
    bool launched = false;
    CK(capture_graphs(c));
    while (c->pending >= 8) {
        HIP_OK(c, hipGraphLaunch(c->graph8, c->stream));
        c->pending -= 8;
        launched = true;
    }
    if (launched) {
        HIP_OK(c, hipMemcpyAsync(c->hs_pin, c->dst, kStateHead, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(c, hipEventRecord(c->ev_status, c->stream));
        c->unchecked = true;
    }
    if (c->unchecked && hipEventQuery(c->ev_status) == hipSuccess) {
        DevState hs;
        std::memcpy(&hs, c->hs_pin, kStateHead);
        CK(ctx_state_status(c, hs));
    }
    return MPH_OK;
}

int mph_set_step_batching(MphCtx* c, int on)
{
    if (!c) return MPH_ERR_ARG;
    if (c->dist) return on ? fail(c, MPH_ERR_ARG, "step batching is not available in slab mode") : MPH_OK;
    HIP_OK(c, hipSetDevice(c->device));
    if (!on) {
        c->batch_steps = false;
        return ctx_flush(c);
    }
    if (!c->hs_pin) HIP_OK(c, hipHostMalloc(&c->hs_pin, kStateHead, hipHostMallocDefault));
    if (!c->ev_status) HIP_OK(c, hipEventCreateWithFlags(&c->ev_status, hipEventDisableTiming));
    c->batch_steps = true;
    return MPH_OK;
}

int mph_step(MphCtx* c, int nsteps)
{
    if (!c || nsteps < 0) return MPH_ERR_ARG;
    HIP_OK(c, hipSetDevice(c->device));
    if (c->dist) return dist_step(c, nsteps);
    if (nsteps == 0 || c->n == 0) {
        for (int k = 0; k < nsteps; ++k) c->time += c->cfg.dt;
        return MPH_OK;
    }
    if (c->batch_steps && !c->phase_timing) return step_batched(c, nsteps);
    CK(ctx_flush(c));
    int left = nsteps;
    if (c->phase_timing) {
        // the graphs' batches (8 steps, then single steps; the output-only stores on each batch's
        // last step) as direct launches with the phase events (HIP cannot time events recorded
        // inside a captured graph), read after every batch
        while (left > 0) {
            const int b = left >= 8 ? 8 : 1;
            for (int k = 0; k < b; ++k) enqueue_step(c->L, k == b - 1, c->ev8.data() + 3 * k);
            HIP_OK(c, hipGetLastError());
            CK(accumulate_phases(c, c->ev8, b));
            left -= b;
        }
    } else {
        CK(capture_graphs(c));
        while (left >= 8) { HIP_OK(c, hipGraphLaunch(c->graph8, c->stream)); left -= 8; }
        CK(launch_singles(c, left));
    }
    for (int k = 0; k < nsteps; ++k) c->time += c->cfg.dt;
    c->stepped = true;
    // the error flags, copied into pinned memory behind the steps (a pageable copy is staged by the
    // runtime).  Polling the stream instead of the blocking wait measured the same per call
    // (profiles/r05/sync_path/).
    if (!c->hs_pin) HIP_OK(c, hipHostMalloc(&c->hs_pin, kStateHead, hipHostMallocDefault));
    HIP_OK(c, hipMemcpyAsync(c->hs_pin, c->dst, kStateHead, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    DevState hs;
    std::memcpy(&hs, c->hs_pin, kStateHead);
    CK(ctx_state_status(c, hs));
    return MPH_OK;
}

int mph_synchronize(MphCtx* c)
{
    if (!c) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    // slab mode: the second stream too (halo, face pass B, early send, elastic ghost exchanges)
    if (c->dist && c->dist->stream2) HIP_OK(c, hipStreamSynchronize(c->dist->stream2));
    return MPH_OK;
}

int mph_particle_count(const MphCtx* c) { return c ? c->n_glob : -1; }
double mph_time(const MphCtx* c) { return c ? c->time : 0.0; }
const char* mph_last_error(const MphCtx* c) { return c ? c->err.c_str() : g_create_error.c_str(); }

int mph_get_scalars(const MphCtx* c, double* out)
{
    if (!c || !out) return MPH_ERR_ARG;
    fill_scalars(c->h, c->cfg, out);
    return MPH_OK;
}

int mph_get(MphCtx* c, int field, void* out)
{
    if (!c || !out) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    HIP_OK(c, hipSetDevice(c->device));
    double* o = (double*)out;
    int* oi = (int*)out;
    // structure rows: every list built here (single context), or the slots this rank computes
    // (slab mode: its owned elastic particles; the lists of ghost slots are partial)
    const int ns = c->dist ? (int)c->sl_s.size() : (int)c->S.orig.size();
    auto sidx = [c](int k) { return c->dist ? c->sl_s[k] : k; };
    // static inputs: every particle, or (slab-local creation) the ones this rank was created with
    const int nin = (int)c->prop.size();
    switch (field) {
    case MPH_FIELD_POSITION: return download_soa3(c, c->B.x, c->B.y, c->B.z, c->B.id, o);
    case MPH_FIELD_VELOCITY: return download_soa3(c, c->B.vx, c->B.vy, c->B.vz, c->B.id, o);
    case MPH_FIELD_INITIAL_POSITION:
        for (int k = 0; k < nin; ++k) std::memcpy(o + 3 * (size_t)glob_id(c, k), &c->pos0[3 * (size_t)k], 3 * sizeof(double));
        return MPH_OK;
    case MPH_FIELD_FORCE: return download_vec(c, c->force, c->A.id, o, 3);
    case MPH_FIELD_ACCELERATION: return download_vec(c, c->acc, c->A.id, o, 3);
    case MPH_FIELD_GRAVITY_CENTER: return download_soa3(c, c->gx, c->gy, c->gz, c->A.id, o);
    case MPH_FIELD_PRESSURE_P: return download_scalar(c, c->pres, c->A.id, o);
    case MPH_FIELD_PRESSURE_A: return download_scalar(c, c->pa, c->A.id, o);
    case MPH_FIELD_DENSITY_A: return download_scalar(c, c->dens_a, c->A.id, o);
    case MPH_FIELD_VOL_STRAIN_P: return download_scalar(c, c->vstrain, c->A.id, o);
    case MPH_FIELD_DIVERGENCE_P: return download_scalar(c, c->divp, c->A.id, o);
    case MPH_FIELD_NEIGHBOR_COUNT: return download_scalar(c, c->nbcount, c->A.id, oi);
    case MPH_FIELD_MASS:
        for (int k = 0; k < nin; ++k) o[glob_id(c, k)] = c->cfg.density[c->prop[k]] * c->h.vol;
        return MPH_OK;
    case MPH_FIELD_KAPPA: {
        // initializeFluid (1317-1319) before the first step, calculatePhysicalCoefficients after
        std::vector<double> vs(c->stepped ? (size_t)c->n_glob : 0, 0.0);
        if (c->stepped) CK(download_scalar(c, c->vstrain, c->A.id, vs.data()));
        for (int k = 0; k < nin; ++k) {
            const int i = glob_id(c, k);
            o[i] = (c->stepped && vs[i] < 0.0) ? 0.0 : c->cfg.bulk_modulus[c->prop[k]];
        }
        return MPH_OK;
    }
    case MPH_FIELD_LAMBDA:
        for (int k = 0; k < nin; ++k) o[glob_id(c, k)] = c->cfg.bulk_viscosity[c->prop[k]];
        return MPH_OK;
    case MPH_FIELD_MU:
        for (int k = 0; k < nin; ++k) o[glob_id(c, k)] = c->cfg.shear_viscosity[c->prop[k]];
        return MPH_OK;
    case MPH_FIELD_PROPERTY:
        for (int k = 0; k < nin; ++k) oi[glob_id(c, k)] = c->prop[k];
        return MPH_OK;
    case MPH_FIELD_INITIAL_STRUCTURE_NEIGHBOR_COUNT:
        for (int k = 0; k < nin; ++k) oi[glob_id(c, k)] = 0;
        for (int k = 0; k < ns; ++k) oi[glob_id(c, c->S.orig[sidx(k)])] = c->S.count[sidx(k)];
        return MPH_OK;
    case MPH_FIELD_DEFORM_GRADIENT: return download_struct_m33(c, c->Sd.F, o);
    case MPH_FIELD_STRAIN: return download_struct_m33(c, c->Sd.E, o);
    case MPH_FIELD_STRESS: return download_struct_m33(c, c->Sd.S, o);
    case MPH_FIELD_NORMALIZER:
        for (int k = 0; k < nin; ++k) std::memset(o + (size_t)9 * glob_id(c, k), 0, sizeof(double) * 9);
        for (int k = 0; k < ns; ++k)
            std::memcpy(o + (size_t)9 * glob_id(c, c->S.orig[sidx(k)]), &c->S.normalizer[(size_t)9 * sidx(k)],
                        sizeof(double) * 9);
        return MPH_OK;
    case MPH_FIELD_VIRIAL_STRESS:
    case MPH_FIELD_VIRIAL_PRESSURE: {
        const int w = field == MPH_FIELD_VIRIAL_STRESS ? 9 : 1;
        std::memset(o, 0, sizeof(double) * w * (size_t)c->n_glob);
        if (!c->vir) return MPH_OK;   // never computed (the reference's array is uninitialised)
        std::vector<double> h((size_t)w * c->n);
        std::vector<int> id(c->n);
        HIP_OK(c, hipMemcpyAsync(h.data(), w == 9 ? c->vir : c->vpres, sizeof(double) * w * c->n,
                                 hipMemcpyDeviceToHost, c->stream));
        HIP_OK(c, hipMemcpyAsync(id.data(), c->A.id, sizeof(int) * c->n, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(c, hipStreamSynchronize(c->stream));
        for (int i = 0; i < c->n; ++i)
            if (id[i] >= 0) std::memcpy(o + (size_t)w * id[i], &h[(size_t)w * i], sizeof(double) * w);
        return MPH_OK;
    }
    case MPH_FIELD_LAMBDA_LAMES:
    case MPH_FIELD_MU_LAMES:
        for (int k = 0; k < nin; ++k) o[glob_id(c, k)] = 0.0;
        for (int k = 0; k < ns; ++k)
            o[glob_id(c, c->S.orig[sidx(k)])] =
                field == MPH_FIELD_LAMBDA_LAMES ? c->S.lame_l[sidx(k)] : c->S.lame_m[sidx(k)];
        return MPH_OK;
    default: return fail(c, MPH_ERR_ARG, "unknown field " + std::to_string(field));
    }
}

int mph_compute_virial(MphCtx* c)
{
    if (!c) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    HIP_OK(c, hipSetDevice(c->device));
    if (!c->vir) {
        // slab mode: the array capacity (c->P.n), the held count changes every step
        const size_t cap = (size_t)std::max(c->dist ? c->P.n : c->n, 1);
        CK(dalloc(c, &c->vir, 9 * cap));
        CK(dalloc(c, &c->vpres, cap));
    }
    if (c->dist) return dist_virial(c);
    // after a step the integrated state B is in A (list) order; before the first step A is current
    if (c->phase_timing) HIP_OK(c, hipEventRecord(c->ev_vir[0], c->stream));
    CK(virial_full_lists(c));
    launch_virial(c->L, c->stepped ? c->B : c->A, c->vir, c->vpres);
    HIP_OK(c, hipGetLastError());
    if (c->phase_timing) HIP_OK(c, hipEventRecord(c->ev_vir[1], c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    if (c->phase_timing) {
        float ms = 0.0f;
        HIP_OK(c, hipEventElapsedTime(&ms, c->ev_vir[0], c->ev_vir[1]));
        c->phase_ms[2] += ms;
    }
    return MPH_OK;
}

int mph_set(MphCtx* c, int field, const void* in)
{
    if (!c || !in) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    if (field != MPH_FIELD_POSITION && field != MPH_FIELD_VELOCITY)
        return fail(c, MPH_ERR_ARG, "mph_set supports Position and Velocity");
    HIP_OK(c, hipSetDevice(c->device));
    const int n = c->n;
    const double* v = (const double*)in;
    // current state lives in the B set in the order of B.id: rewrite it in that order
    std::vector<double> h(n);
    std::vector<int> id(n);
    HIP_OK(c, hipMemcpy(id.data(), c->B.id, sizeof(int) * n, hipMemcpyDeviceToHost));
    double* dst[3] = {c->B.x, c->B.y, c->B.z};
    if (field == MPH_FIELD_VELOCITY) { dst[0] = c->B.vx; dst[1] = c->B.vy; dst[2] = c->B.vz; }
    for (int k = 0; k < 3; ++k) {
        for (int i = 0; i < n; ++i) h[i] = id[i] >= 0 ? v[3 * (size_t)id[i] + k] : 0.0;
        HIP_OK(c, hipMemcpy(dst[k], h.data(), sizeof(double) * n, hipMemcpyHostToDevice));
    }
    return MPH_OK;
}

int mph_set_initial_velocity_profile(MphCtx* c)
{
    if (!c) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    HIP_OK(c, hipSetDevice(c->device));
    const size_t n = (size_t)c->n_glob;
    // slab mode: mph_get fills the owned entries and mph_set writes only those back
    std::vector<double> pos(3 * n, 0.0), vel(3 * n, 0.0);
    CK(mph_get(c, MPH_FIELD_POSITION, pos.data()));
    CK(mph_get(c, MPH_FIELD_VELOCITY, vel.data()));
    // the static inputs this context holds, with the current state of the same particles
    const int nin = (int)c->prop.size();
    std::vector<double> p(3 * (size_t)nin), v(3 * (size_t)nin);
    for (int k = 0; k < nin; ++k)
        for (int d = 0; d < 3; ++d) {
            p[3 * (size_t)k + d] = pos[3 * (size_t)glob_id(c, k) + d];
            v[3 * (size_t)k + d] = vel[3 * (size_t)glob_id(c, k) + d];
        }
    CK(mph_velocity_profile_arrays(&c->cfg, c->time, nin, c->prop.data(), p.data(), c->pos0.data(), v.data()));
    for (int k = 0; k < nin; ++k)
        for (int d = 0; d < 3; ++d) vel[3 * (size_t)glob_id(c, k) + d] = v[3 * (size_t)k + d];
    return mph_set(c, MPH_FIELD_VELOCITY, vel.data());
}

int mph_write_prof(MphCtx* c, const char* path)
{
    if (!c || !path) return MPH_ERR_ARG;
    if (c->dist) return dist_write_output(c, path, kOutProf);   // collective; rank 0 writes
    const int n = c->n_glob;
    std::vector<double> pos(3 * (size_t)n), vel(3 * (size_t)n);
    CK(mph_get(c, MPH_FIELD_POSITION, pos.data()));
    CK(mph_get(c, MPH_FIELD_VELOCITY, vel.data()));
    return mph_write_prof_arrays(path, &c->cfg, c->time, n, c->prop.data(), pos.data(), c->pos0.data(),
                                 vel.data());
}

static int write_vtk_any(MphCtx* c, const char* path, bool xml)
{
    if (!c || !path) return MPH_ERR_ARG;
    if (c->dist) return dist_write_output(c, path, xml ? kOutVtu : kOutVtk);   // collective; rank 0 writes
    const size_t n = (size_t)c->n_glob;
    std::vector<double> pos(3 * n), vel(3 * n), acc(3 * n), force(3 * n), stress(9 * n), strain(9 * n);
    std::vector<int> isnc(n), nc(n);
    CK(mph_get(c, MPH_FIELD_POSITION, pos.data()));
    CK(mph_get(c, MPH_FIELD_VELOCITY, vel.data()));
    CK(mph_get(c, MPH_FIELD_ACCELERATION, acc.data()));
    CK(mph_get(c, MPH_FIELD_FORCE, force.data()));
    CK(mph_get(c, MPH_FIELD_STRESS, stress.data()));
    CK(mph_get(c, MPH_FIELD_STRAIN, strain.data()));
    CK(mph_get(c, MPH_FIELD_INITIAL_STRUCTURE_NEIGHBOR_COUNT, isnc.data()));
    CK(mph_get(c, MPH_FIELD_NEIGHBOR_COUNT, nc.data()));
    auto writer = xml ? mph_write_vtu_arrays : mph_write_vtk_arrays;
    return writer(path, c->n_glob, c->prop.data(), pos.data(), c->pos0.data(), vel.data(), acc.data(), force.data(),
                  stress.data(), strain.data(), isnc.data(), nc.data());
}

int mph_write_vtk(MphCtx* c, const char* path) { return write_vtk_any(c, path, false); }

int mph_write_vtu(MphCtx* c, const char* path) { return write_vtk_any(c, path, true); }

int mph_output_wait(MphCtx* c)
{
    if (!c) return MPH_ERR_ARG;
    if (c->out_thread.joinable()) c->out_thread.join();
    const int rc = c->out_rc;
    c->out_rc = MPH_OK;
    if (rc) return fail(c, rc, "asynchronous .vtk write failed");
    return MPH_OK;
}

int mph_write_vtk_async(MphCtx* c, const char* path)
{
    if (!c || !path) return MPH_ERR_ARG;
    CK(mph_output_wait(c));   // at most one file in flight
    if (c->dist) return dist_write_output(c, path, kOutVtkAsync);   // collective; rank 0 formats and writes
    struct Snap {
        std::string path;
        std::vector<double> pos, pos0, vel, acc, force, stress, strain;
        std::vector<int> prop, isnc, nc;
    };
    const size_t n = (size_t)c->n_glob;
    auto s = std::make_shared<Snap>();
    s->path = path;
    s->pos.resize(3 * n); s->vel.resize(3 * n); s->acc.resize(3 * n); s->force.resize(3 * n);
    s->stress.resize(9 * n); s->strain.resize(9 * n); s->isnc.resize(n); s->nc.resize(n);
    s->pos0 = c->pos0;
    s->prop = c->prop;
    CK(mph_get(c, MPH_FIELD_POSITION, s->pos.data()));
    CK(mph_get(c, MPH_FIELD_VELOCITY, s->vel.data()));
    CK(mph_get(c, MPH_FIELD_ACCELERATION, s->acc.data()));
    CK(mph_get(c, MPH_FIELD_FORCE, s->force.data()));
    CK(mph_get(c, MPH_FIELD_STRESS, s->stress.data()));
    CK(mph_get(c, MPH_FIELD_STRAIN, s->strain.data()));
    CK(mph_get(c, MPH_FIELD_INITIAL_STRUCTURE_NEIGHBOR_COUNT, s->isnc.data()));
    CK(mph_get(c, MPH_FIELD_NEIGHBOR_COUNT, s->nc.data()));
    const int nn = c->n_glob;
    c->out_thread = std::thread([c, s, nn] {
        c->out_rc = mph_write_vtk_arrays(s->path.c_str(), nn, s->prop.data(), s->pos.data(), s->pos0.data(),
                                         s->vel.data(), s->acc.data(), s->force.data(), s->stress.data(),
                                         s->strain.data(), s->isnc.data(), s->nc.data());
    });
    return MPH_OK;
}

int mph_phase_timing(MphCtx* c, int on)
{
    if (!c) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    if (c->dist) return on ? fail(c, MPH_ERR_ARG, "phase timing is not available in slab mode") : MPH_OK;
    HIP_OK(c, hipSetDevice(c->device));
    const bool want = on != 0;
    if (want == c->phase_timing) return MPH_OK;
    HIP_OK(c, hipStreamSynchronize(c->stream));
    c->phase_timing = want;   // (mph_step then launches directly; the graphs stay for later)
    if (want && c->ev_vir.empty()) {
        c->ev_vir.assign(2, nullptr);
        for (auto& e : c->ev_vir) HIP_OK(c, hipEventCreate(&e));
        c->ev8.assign(3 * 8, nullptr);
        for (auto& e : c->ev8) HIP_OK(c, hipEventCreate(&e));
    }
    return MPH_OK;
}

int mph_phase_times(const MphCtx* c, double* out3)
{
    if (!c || !out3) return MPH_ERR_ARG;
    for (int k = 0; k < 3; ++k) out3[k] = c->phase_ms[k];
    return MPH_OK;
}

int mph_profile_steps(MphCtx* c, int nsteps, double* avg_ms, int* launches, char* names32)
{
    if (!c || nsteps <= 0 || !avg_ms || !launches || !names32) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    HIP_OK(c, hipSetDevice(c->device));
    EventProfiler prof;
    if (c->dist) {
        CK(dist_step(c, nsteps, &prof));
    } else {
        Launch L = c->L;
        L.prof = &prof;
        for (int k = 0; k < nsteps; ++k) enqueue_step(L, k == nsteps - 1);
        HIP_OK(c, hipGetLastError());
        HIP_OK(c, hipStreamSynchronize(c->stream));
        for (int k = 0; k < nsteps; ++k) c->time += c->cfg.dt;
        c->stepped = true;
    }
    std::vector<std::string> order;
    std::map<std::string, std::pair<double, int>> acc;
    // the kernels' intervals from the first event on, for their union (kernels of the two streams
    // of a slab step run concurrently, so the sum of their times overstates the GPU time)
    std::vector<std::pair<float, float>> span;
    for (auto& r : prof.recs) {
        float ms = 0.0f, t0 = 0.0f;
        HIP_OK(c, hipEventElapsedTime(&ms, r.a, r.b));
        HIP_OK(c, hipEventElapsedTime(&t0, prof.recs[0].a, r.a));
        if (r.floor >= 0) {
            float tf = 0.0f;
            HIP_OK(c, hipEventElapsedTime(&tf, prof.recs[0].a, prof.floors[r.floor]));
            if (tf > t0) {
                ms = std::max(0.0f, ms - (tf - t0));
                t0 = tf;
            }
        }
        span.emplace_back(t0, t0 + ms);
        if (!acc.count(r.name)) order.push_back(r.name);
        acc[r.name].first += ms;
        acc[r.name].second += 1;
    }
    std::sort(span.begin(), span.end());
    double busy = 0.0, hi = -1e30;
    for (auto& iv : span) {
        if (iv.first > hi) { busy += iv.second - iv.first; hi = iv.second; }
        else if (iv.second > hi) { busy += iv.second - hi; hi = iv.second; }
    }
    int k = 0;
    for (auto& name : order) {
        if (k >= MPH_PROFILE_MAX - 1) break;
        avg_ms[k] = acc[name].first / acc[name].second;
        launches[k] = acc[name].second;
        std::snprintf(names32 + 32 * k, 32, "%s", name.c_str());
        ++k;
    }
    // last entry: "gpu_busy", the union of the kernel intervals per step (launches = steps)
    avg_ms[k] = busy / nsteps;
    launches[k] = nsteps;
    std::snprintf(names32 + 32 * k, 32, "%s", "gpu_busy");
    ++k;
    DevState hs;
    HIP_OK(c, hipMemcpy(&hs, c->dst, kStateHead, hipMemcpyDeviceToHost));
    CK(ctx_state_status(c, hs));
    return k;
}

// The list kernels as the timed steps run them: each one captured `reps` times into a graph of
// its own (the output-only stores on every 8th, as in the 8-step graph), replayed once to warm,
// then once between two HIP events.  Each replay recomputes what the last step left (the lists,
// pass A's products, B from A), bit for bit, so the state does not change; pass B is skipped with
// elastic slots (the substeps after it have moved them in B).  Slab contexts: the same on the
// rank's local set, pass B as its single launch and before pass A (whose replay clears the
// ghosts' halo pressure in the pass-B records until the next step's halo).  Needs one step done.
int mph_profile_graphs(MphCtx* c, int reps, double* avg_ms3)
{
    if (!c || reps <= 0 || reps > 64 || !avg_ms3) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    if (!c->stepped) return ctx_fail(c, MPH_ERR_ARG, "mph_profile_graphs: run a step first");
    HIP_OK(c, hipSetDevice(c->device));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIP_OK(c, hipEventCreate(&e0));
    HIP_OK(c, hipEventCreate(&e1));
    int rc = MPH_OK;
    for (int k = 0; k < 3; ++k) avg_ms3[k] = -1.0;
    // pass B before pass A: in slab mode pass A zeroes the pressure of the ghosts' pass-B records,
    // which the halo had filled (the next step's halo fills them again)
    for (int kk = 0; kk < 3 && rc == MPH_OK; ++kk) {
        const int k = kk == 0 ? 0 : (kk == 1 ? 2 : 1);
        if (k == 2 && c->P.n_struct > 0) continue;
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        bool ok = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
        if (ok) {
            for (int r = 0; r < reps; ++r) {
                const bool last = r % 8 == 7 || r == reps - 1;
                Launch La = c->L;
                if (c->dist) La.wface = c->dist->wface;   // slab mode: pass B in one launch (phase 0)
                if (!last) {
                    La.dens_a = La.vstrain = La.divp = nullptr;
                    if (!c->P.surface) La.gx = La.gy = La.gz = La.pa = nullptr;
                    La.force = La.acc = nullptr;
                }
                if (k == 0) launch_neighbors(La);
                else if (k == 1) launch_pass_a(La);
                else launch_pass_b(La);
            }
            ok = hipStreamEndCapture(c->stream, &g) == hipSuccess && g;
        }
        ok = ok && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess;
        if (g) (void)hipGraphDestroy(g);
        float ms = 0.0f;
        ok = ok && hipGraphUpload(ge, c->stream) == hipSuccess && hipGraphLaunch(ge, c->stream) == hipSuccess &&
             hipEventRecord(e0, c->stream) == hipSuccess && hipGraphLaunch(ge, c->stream) == hipSuccess &&
             hipEventRecord(e1, c->stream) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
             hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
        if (ge) (void)hipGraphExecDestroy(ge);
        if (ok) avg_ms3[k] = ms / reps;
        else rc = ctx_fail(c, MPH_ERR_HIP, "mph_profile_graphs: graph capture or replay failed");
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    CK(rc);
    HIP_OK(c, hipStreamSynchronize(c->stream));
    DevState hs;
    HIP_OK(c, hipMemcpy(&hs, c->dst, kStateHead, hipMemcpyDeviceToHost));
    return ctx_state_status(c, hs);
}

int mph_neighbor_stats(MphCtx* c, double* mean, int* mx)
{
    if (!c || !mean || !mx) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    HIP_OK(c, hipSetDevice(c->device));
    // NeighborCount of the particles held here (slab mode: owned + ghosts), reduced on the host
    std::vector<int> h(c->n);
    if (c->n) HIP_OK(c, hipMemcpy(h.data(), c->nbcount, sizeof(int) * c->n, hipMemcpyDeviceToHost));
    long long sum = 0;
    int m = 0;
    for (int v : h) { sum += v; m = v > m ? v : m; }
    *mean = c->n ? (double)sum / c->n : 0.0;
    *mx = m;
    return MPH_OK;
}

// The lists' rows as the last search left them (mph_kernels.hip RowMask): per particle (sorted
// order) its rows [0, ncount) and, per wave, the row jumps -- gap k of lane s is the rows
// [byte k of lgap[s], byte k of lhdr[s >> 6]) for k below the jump count in byte 7 of the header.
struct HostRows {
    std::vector<int> rows;
    std::vector<unsigned long long> hdr, gap;
    // whether row r of particle s holds one of its entries
    bool ok(int s, int r) const
    {
        const unsigned long long h = hdr[s >> 6];
        const int J = (int)(h >> 56);
        for (int k = 0; k < J; ++k) {
            const int a = (int)((gap[s] >> (8 * k)) & 0xff), b = (int)((h >> (8 * k)) & 0xff);
            if (r >= a && r < b) return false;
        }
        return r < rows[s];
    }
    int entries(int s) const
    {
        const unsigned long long h = hdr[s >> 6];
        const int J = (int)(h >> 56);
        int e = std::min(rows[s], kTileRows);
        for (int k = 0; k < J; ++k) e -= (int)((h >> (8 * k)) & 0xff) - (int)((gap[s] >> (8 * k)) & 0xff);
        return e;
    }
};

static int host_rows(MphCtx* c, HostRows& R)
{
    const int n = c->n;
    const size_t ntile = ((size_t)n + kTile - 1) / kTile;
    R.rows.resize(n);
    R.hdr.resize(ntile);
    R.gap.resize(ntile * kTile);
    if (!n) return MPH_OK;
    HIP_OK(c, hipMemcpy(R.rows.data(), c->ncount, sizeof(int) * n, hipMemcpyDeviceToHost));
    HIP_OK(c, hipMemcpy(R.hdr.data(), c->lhdr, sizeof(unsigned long long) * ntile, hipMemcpyDeviceToHost));
    HIP_OK(c, hipMemcpy(R.gap.data(), c->lgap, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
    return MPH_OK;
}

int mph_list_stats(MphCtx* c, double* mean, int* mx)
{
    if (!c || !mean || !mx) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    HIP_OK(c, hipSetDevice(c->device));
    HostRows R;   // stored list lengths (the rows outside the gaps), reduced on the host
    CK(host_rows(c, R));
    std::vector<int> h(c->n);
    for (int s = 0; s < c->n; ++s) h[s] = R.entries(s);
    long long sum = 0;
    int m = 0;
    for (int v : h) { sum += v; m = v > m ? v : m; }
    *mean = c->n ? (double)sum / c->n : 0.0;
    *mx = m;
    return MPH_OK;
}

int mph_neighbor_rows(MphCtx* c, int first, int count, int* counts, int* ids, long long ids_cap)
{
    if (!c || first < 0 || count < 0 || !counts || (!ids && ids_cap > 0)) return MPH_ERR_ARG;
    CK(ctx_flush(c));
    if (c->dist) return fail(c, MPH_ERR_UNSUPPORTED, "mph_neighbor_rows: single contexts only");
    if ((long long)first + count > c->n) return fail(c, MPH_ERR_ARG, "mph_neighbor_rows: range past the particle count");
    if (!count) return 0;
    HIP_OK(c, hipSetDevice(c->device));
    const int n = c->n;
    if (c->P.rlf < 3.0e38f)
        return fail(c, MPH_ERR_UNSUPPORTED, "mph_neighbor_rows: the lists keep only the pairs within the passes' "
                                            "radius (create the context with MPH_LIST_FULL=1 for the reference's lists)");
    // the last search's rows are in its sorted order A: A.id maps a row (and an entry) back to the
    // original index, ncount holds the list's length and nbcount NeighborCount in the same order
    std::vector<int> id(n), nv(n);
    HIP_OK(c, hipMemcpy(id.data(), c->A.id, sizeof(int) * n, hipMemcpyDeviceToHost));
    HIP_OK(c, hipMemcpy(nv.data(), c->nbcount, sizeof(int) * n, hipMemcpyDeviceToHost));
    HostRows R;
    CK(host_rows(c, R));
    const std::vector<int>& nc = R.rows;
    std::vector<int> row_of(count, -1);
    for (int s = 0; s < n; ++s)
        if (id[s] >= first && id[s] < first + count) row_of[id[s] - first] = s;
    long long total = 0;
    for (int k = 0; k < count; ++k) {
        if (row_of[k] < 0) return fail(c, MPH_ERR_HIP, "mph_neighbor_rows: particle missing from the sorted set");
        counts[k] = nv[row_of[k]];
        total += std::min(counts[k], kMaxNeighbor);
    }
    if (total > ids_cap) return fail(c, MPH_ERR_ARG, "mph_neighbor_rows: ids_cap too small (" + std::to_string(total) + " needed)");
    // every ELL tile holding a requested row, down to the longest row of its lanes (entry k of lane l
    // at [k][l], 64 ints per entry: one contiguous copy per tile)
    std::map<int, std::vector<int>> tiles;
    for (int k = 0; k < count; ++k) {
        const int t = row_of[k] >> 6;
        if (tiles.count(t)) continue;
        int m = 0;
        for (int s = t * kTile; s < std::min(n, (t + 1) * kTile); ++s) m = std::max(m, std::min(nc[s], kTileRows));
        std::vector<int>& buf = tiles[t];
        buf.resize((size_t)m * kTile);
        if (m) HIP_OK(c, hipMemcpy(buf.data(), c->nbr + (size_t)t * kTileStride, sizeof(int) * buf.size(),
                                   hipMemcpyDeviceToHost));
    }
    long long w = 0;
    for (int k = 0; k < count; ++k) {
        const int s = row_of[k], m = std::min(counts[k], kMaxNeighbor), rows = std::min(nc[s], kTileRows);
        const std::vector<int>& buf = tiles[s >> 6];
        int q = 0;
        for (int e = 0; e < rows; ++e) {
            if (!R.ok(s, e)) continue;   // a gap of the row jumps
            const int v = buf[(size_t)ell_slot(e, s & 63)];
            const int j = v & kIndexMask;
            if (j >= n || q >= m) return fail(c, MPH_ERR_HIP, "mph_neighbor_rows: list entry past the particle count");
            ids[w + q++] = id[j];
        }
        if (q != m) return fail(c, MPH_ERR_HIP, "mph_neighbor_rows: list rows disagree with NeighborCount");
        std::sort(ids + w, ids + w + m);
        w += m;
    }
    return (int)std::min<long long>(w, 0x7fffffff);
}

void mph_destroy(MphCtx* c)
{
    if (!c) return;
    if (c->out_thread.joinable()) c->out_thread.join();
    (void)hipSetDevice(c->device);
    (void)ctx_flush(c);   // steps accepted under batching still run (their errors are dropped)
    if (c->hs_pin) (void)hipHostFree(c->hs_pin);
    if (c->ev_status) (void)hipEventDestroy(c->ev_status);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->graph1) (void)hipGraphExecDestroy(c->graph1);
    if (c->graph1t) (void)hipGraphExecDestroy(c->graph1t);
    if (c->graph8) (void)hipGraphExecDestroy(c->graph8);
    for (auto* v : {&c->ev8, &c->ev_vir})
        for (hipEvent_t e : *v) (void)hipEventDestroy(e);
    if (c->dist) dist_free(c);
    for (void* p : c->allocs) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

}  // extern "C"

// ---- multi-GPU slab decomposition: see mph_dist.hip ------------------------------------------
