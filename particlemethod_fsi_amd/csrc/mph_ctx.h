// mph_ctx.h -- the device context behind the C ABI (include/mph_gpu.h), shared by the single-GPU
// implementation (mph_ctx.hip) and the slab-decomposed multi-GPU step (mph_dist.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "mph_internal.h"
#include "mph_kernels.h"

// Multi-GPU state of one rank (one process per GPU).  Local particle arrays hold
// [owned | ghosts] in cell order; see mph_dist.hip for the step protocol.
struct MphDist {
    int rank = 0, nranks = 1, left = 0, right = 0;
    mph::SlabGeom g{};
    std::vector<double> cuts;     // interior slab boundaries (MphSlabOptions.cuts); empty: equal widths
    int cap = 0;                  // capacity of every local per-particle array
    int n_own = 0;                // owned particles after the last redistribution (host mirror)
    // Every size of a step lives on the device (DistLayout), so a step has no host round trip and
    // the RCCL transport replays whole steps from captured graphs.  Messages travel with fixed
    // capacities (particles) per direction; a pair of neighbours derives the same capacity for
    // its shared direction from the same counts (send of one = receive of the other).
    mph::DistLayout* lay = nullptr;    // device
    mph::DistLayout* hlay = nullptr;   // pinned host mirror (read after a step batch)
    int cap_sl = 0, cap_sr = 0, cap_rl = 0, cap_rr = 0;
    size_t region = 0;            // bytes of each of the four message buffers
    mph::Soa C;                   // redistributed state (pre-sort order)
    int* cls = nullptr;           // class of every B entry
    // the kept entries of C stay in B (VSrc: C holds the received tail only, vidx[v] = where
    // entry v lives in B); MPH_SLAB_VIRTUAL_C=0 copies them into C
    int* vidx = nullptr;
    bool virt = !(std::getenv("MPH_SLAB_VIRTUAL_C") && std::string(std::getenv("MPH_SLAB_VIRTUAL_C")) == "0");
    int* bcnt = nullptr;          // per (class, block) counts -> offsets
    int* boff = nullptr;
    int* bsum = nullptr;
    char *send_l = nullptr, *send_r = nullptr, *recv_l = nullptr, *recv_r = nullptr;  // device, resizable
    hipStream_t stream2 = nullptr;                   // halo exchange beside the inner pass B
    hipEvent_t ev_a = nullptr, ev_h = nullptr;       // pass A done / halo landed
    // transport: RCCL communicator, or a host callback (tests / hosts without RCCL)
    bool rccl = false;
    bool graphs = false;          // steps replayed from captured graphs (RCCL transport)
    // overlap: pass B of the inner particles overlaps the pass-A halo (and the early send below);
    // off: halo, then one pass B over all particles.  MPH_SLAB_OVERLAP=1 / =0 forces the mode;
    // unset (or "auto") the ranks choose it together at creation (overlap_probe, mph_dist.hip): on
    // when the measured exchanges take longer than the split pass B costs over the single one
    bool overlap = false;
    int overlap_mode = [] {
        const char* e = std::getenv("MPH_SLAB_OVERLAP");
        return (e && std::string(e) == "1") ? 1 : ((e && std::string(e) == "0") ? 0 : -1);
    }();
    // the probe's measurements, max over ranks (ms): halo exchange, redistribution exchange (both at
    // their message capacities), pass B split in two launches minus pass B in one; -1: not probed
    double probe_ms[3] = {-1.0, -1.0, -1.0};
    // early send: within a batch of steps, the redistribution messages of the next step leave
    // while the interior pass B of this one runs (no elastic particles; MPH_SLAB_EARLY=0: off)
    bool early = !(std::getenv("MPH_SLAB_EARLY") && std::string(std::getenv("MPH_SLAB_EARLY")) == "0");
    int* wface = nullptr;                             // face-wavefront flags of the last pass B
    hipEvent_t ev_s = nullptr, ev_x = nullptr;       // early messages packed / exchanged
    char uid[128] = {0};          // ncclUniqueId
    void* comm = nullptr;         // ncclComm_t
    mph_host_exchange_fn host_fn = nullptr;
    void* host_user = nullptr;
    char* host_stage = nullptr;   // pinned staging for the host transport (4 messages)
    // the last host-staged exchange's copies into the device (they read host_stage): the next
    // exchange, possibly on the other stream, waits for them before the callback refills it
    hipEvent_t ev_stage = nullptr;
    bool stage_busy = false;
    // elastic ghost slots (static): local slot indices sent to / received from each neighbour
    int *ss_l = nullptr, *ss_r = nullptr, *sr_l = nullptr, *sr_r = nullptr;
    int nss_l = 0, nss_r = 0, nsr_l = 0, nsr_r = 0;
};

struct MphCtx {
    int device = 0;
    int n = 0;                   // particles held on the device (single GPU: all; slab: owned+ghosts)
    int n_glob = 0;              // particles of the whole problem (length of mph_get arrays)
    MphConfig cfg{};
    mph::HostDerived h{};
    mph::DevParams P{};
    mph::DevTables T{};
    std::string err;
    std::thread out_thread;      // mph_write_vtk_async: the file of the previous output step
    int out_rc = 0;
    double time = 0.0;           // host mirror of Time (same additions as the device)
    bool stepped = false;
    hipStream_t stream = nullptr;
    hipGraphExec_t graph1 = nullptr, graph8 = nullptr;
    hipGraphExec_t graph1t = nullptr;   // one step without the output-only stores (single context)
    // step batching (mph_set_step_batching): single mph_step calls accumulate into 8-step graphs;
    // `pending` steps are accepted but not launched yet, `unchecked`: batches launched whose error
    // flags have not been read; the flags of the last launched batch land in hs_pin (pinned)
    bool batch_steps = false;
    int pending = 0;
    bool unchecked = false;
    void* hs_pin = nullptr;
    hipEvent_t ev_status = nullptr;
    // phase timing (mph_phase_timing): steps launched directly (no graph) with events at every
    // step's phase boundaries -- before the sort, after the search, after the elastic substeps --
    // three per step of a batch of up to 8 (ev8), and around the virial (ev_vir)
    bool phase_timing = false;
    std::vector<hipEvent_t> ev8, ev_vir;
    double phase_ms[3] = {0.0, 0.0, 0.0};   // neighbour search, explicit calculation, virial
    // host copies of the static inputs: original order, or -- slab-local creation -- the
    // particles this rank was created with, whose original indices are gid (ascending)
    std::vector<int> prop;
    std::vector<double> pos0;
    std::vector<int> gid;
    mph::StructureInit S;
    std::vector<int> sl_orig;    // local structure slot -> original particle index
    std::vector<int> sl_s;       // local structure slot -> index into S (the lists built here)
    // device
    mph::DevTables* dT = nullptr;
    mph::DevState* dst = nullptr;
    mph::Soa A, B;               // sorted current state / integrated state (see mph_kernels.h)
    int* rank_of = nullptr;
    int *key = nullptr, *slot = nullptr, *tmp = nullptr, *cnt = nullptr, *start = nullptr, *bsum = nullptr;
    double *vir = nullptr, *vpres = nullptr;   // VirialStress [cap][9] / VirialPressure (A order), lazy
    int *nbr = nullptr, *ncount = nullptr, *nbcount = nullptr;   // list rows / NeighborCount
    unsigned long long *lhdr = nullptr, *lgap = nullptr;          // the lists' row jumps (RowMask)
    double *pres = nullptr, *gx = nullptr, *gy = nullptr, *gz = nullptr, *pa = nullptr;
    double4 *force = nullptr, *acc = nullptr, *fpart = nullptr, *rec = nullptr;
    double *dens_a = nullptr, *vstrain = nullptr, *divp = nullptr;
    mph::StructDev Sd;
    std::vector<void*> allocs;
    mph::Launch L;
    MphDist* dist = nullptr;     // non-null in slab mode
};

namespace mph {

int ctx_fail(MphCtx* c, int code, const std::string& msg);
int ctx_hip_fail(MphCtx* c, hipError_t e, const char* what);
void* ctx_alloc(MphCtx* c, size_t bytes, int* status);

template <typename T>
int ctx_dalloc(MphCtx* c, T** p, size_t count)
{
    int st = MPH_OK;
    *p = (T*)ctx_alloc(c, (count ? count : 1) * sizeof(T), &st);
    return st;
}

void ctx_fill_launch(MphCtx* c);
// cells between a fast-path interior particle and a grid face along axis d: stencil half-width + 1
inline int stencil_margin(const DevParams& P, int d)
{
    const int ca = contig_axis(P.dim, P.perm);
    return (d == ca ? P.sa : kReach) + 1;
}
int ctx_state_status(MphCtx* c, const DevState& hs);   // kernel error flags -> MphStatus

void ctx_set_global_error(const std::string& msg);   // mph_last_error(NULL)
// ids/n_glob: slab-local creation (the arrays hold n of n_glob particles, original indices ids)
int ctx_create(MphCtx** out, const MphConfig* cfg, int n, const int* property, const double* pos,
               const double* pos0, const double* vel, int device, MphDist* dist, const int* ids = nullptr,
               int n_glob = 0);
// original index of host input k (identity unless created slab-local)
inline int glob_id(const MphCtx* c, int k) { return c->gid.empty() ? k : c->gid[k]; }

// slab mode (mph_dist.hip)
int dist_setup(MphCtx* c, const double* pos, std::vector<int>& owned);   // geometry + owned set
// elastic slots of this rank: lsl = [owned | ghosts from the left | ghosts from the right] (global
// slot ids), n_own owned; records the per-substep ghost exchange lists
int dist_struct_setup(MphCtx* c, std::vector<int>& lsl, int& n_own, int& n_inner);
int dist_alloc(MphCtx* c);                                               // exchange buffers
int dist_init(MphCtx* c);                                                // first exchange + init sums
int dist_step(MphCtx* c, int nsteps, Profiler* prof = nullptr);
// host mirror of the layout + error flags after a batch; grows message capacities past 90 %
int dist_sync(MphCtx* c, bool grow_ok = true);
// output in slab mode (collective): every rank's owned records gathered on rank 0, which writes
// `path` with the single-context writers (kind: kOut*); the virial over the owned particles
constexpr int kOutProf = 0, kOutVtk = 1, kOutVtu = 2, kOutVtkAsync = 3;
int dist_write_output(MphCtx* c, const char* path, int kind);
int dist_virial(MphCtx* c);
int virial_full_lists(MphCtx* c);   // the step's lists again with every neighbour (mph_ctx.hip)
void dist_free(MphCtx* c);

}  // namespace mph

#define MPH_HIP_OK(ctx, expr)                                                \
    do {                                                                     \
        hipError_t _e = (expr);                                              \
        if (_e != hipSuccess) return mph::ctx_hip_fail(ctx, _e, #expr);      \
    } while (0)

#define MPH_CK(expr)                   \
    do {                               \
        int _r = (expr);               \
        if (_r != MPH_OK) return _r;   \
    } while (0)
