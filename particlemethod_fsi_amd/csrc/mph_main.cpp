// mph_main.cpp -- `mph_explicit`: drop-in replacement of the reference executable.
//
// Same command line as main.cpp:494-508:
//     mph_explicit <data> <grid> <prof pattern> <vtk pattern> <log> [nthreads] [device]
// Same driver semantics as main.cpp:528-700: read files, initialise, write output.vtk, then
// loop while Time < EndTime + 1e-5*Dt writing the .prof before a step (583-589) and the .vtk
// after a step (672-683).  Differences: the physics runs on MI355X through libmph_gpu.so;
// the .prof holds the current state (the OpenACC build writes stale host arrays);
// the timing report is wall time of the step loop, not clock() CPU time.  A <vtk pattern> ending
// in ".vtu" writes binary VTK XML files instead (mph_write_vtu).
//
// Several GPUs: MPH_SLABS=N runs the same case as N slab ranks (include/mph_gpu.h, one process
// per rank): the process forks N - 1 ranks before any HIP call, rank r takes device
// (device + r) mod the device count (MPH_SLAB_SHARE_DEVICE=1: all on `device`), the slabs lie
// along MPH_SLAB_AXIS (default z in 3-D, x in 2-D), the transport is RCCL (rank 0 makes the unique
// id and hands it to the others through pipes) or, with MPH_SLAB_TRANSPORT=host, neighbour
// exchanges over socket pairs.  Every output call is collective and rank 0 writes the files the
// single-GPU run writes, with the same cadence.
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/prctl.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <roctracer/roctx.h>

#include "../../include/mph_gpu.h"

static FILE* g_log = nullptr;

static bool g_quiet = false;   // slab ranks other than 0 report errors only

static void logf(const char* fmt, ...)
{
    if (g_quiet) return;
    va_list a, b;
    va_start(a, fmt);
    va_copy(b, a);
    if (g_log) vfprintf(g_log, fmt, a);
    vfprintf(stderr, fmt, b);
    va_end(a);
    va_end(b);
    if (g_log) fflush(g_log);
}

// ---- slab ranks: failure propagation ---------------------------------------------------------
// A rank that fails must not leave the others blocked in RCCL (no timeout there) or orphaned on
// their GPUs.  Children die with rank 0 (PR_SET_PDEATHSIG); rank 0 reaps children from a SIGCHLD
// handler and, on any non-zero or abnormal exit, kills the remaining ranks and exits 1 itself --
// from the handler, since rank 0 may be blocked inside a collective with the dead rank.
static constexpr int kMaxRanks = 64;
static pid_t g_child_pid[kMaxRanks];
static volatile sig_atomic_t g_child_done[kMaxRanks];   // 0 running, 1 exited 0, 2 failed
static volatile sig_atomic_t g_nchildren = 0;

static void kill_children()
{
    for (int k = 0; k < g_nchildren; ++k)
        if (g_child_done[k] == 0 && g_child_pid[k] > 0) kill(g_child_pid[k], SIGKILL);
}

static void on_sigchld(int)
{
    // only the registered ranks are reaped: any other child (a library's helper process) keeps its
    // exit status for its owner and cannot end the run
    const int saved = errno;
    for (int k = 0; k < g_nchildren; ++k) {
        if (g_child_done[k] != 0 || g_child_pid[k] <= 0) continue;
        int st = 0;
        if (waitpid(g_child_pid[k], &st, WNOHANG) != g_child_pid[k]) continue;
        const bool ok = WIFEXITED(st) && WEXITSTATUS(st) == 0;
        g_child_done[k] = ok ? 1 : 2;
        if (!ok) {
            static const char msg[] = "error: a slab rank failed; stopping the other ranks\n";
            (void)!write(2, msg, sizeof(msg) - 1);
            kill_children();
            _exit(1);
        }
    }
    errno = saved;
}

static void die(MphCtx* c, int rc, const char* what)
{
    g_quiet = false;
    logf("error: %s failed (%d): %s\n", what, rc, c ? mph_last_error(c) : "");
    kill_children();   // rank 0: the other ranks would wait for it forever (children: none)
    std::exit(1);
}

// ---- slab ranks: fork, socket-pair ring, RCCL id over pipes ----------------------------------

struct SlabRank {
    int rank = 0, nranks = 1;
    int left_fd = -1, right_fd = -1;   // host transport: the ring links to the two neighbours
    int uid_fd = -1;                   // RCCL: rank > 0 reads the unique id here
    std::vector<int> uid_out;          // rank 0 writes it to these
    std::vector<pid_t> children;
};

static bool write_all(int fd, const void* p, size_t n)
{
    const char* c = (const char*)p;
    while (n) {
        const ssize_t k = write(fd, c, n);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

static bool read_all(int fd, void* p, size_t n)
{
    char* c = (char*)p;
    while (n) {
        const ssize_t k = read(fd, c, n);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

// mph_host_exchange_fn over the two ring sockets: all four transfers progress together (poll), so
// two neighbours sending large messages to each other cannot block on full socket buffers
static int socket_exchange(void* user, const void* send_l, size_t bsl, const void* send_r, size_t bsr,
                           void* recv_l, size_t brl, void* recv_r, size_t brr)
{
    const SlabRank& R = *(const SlabRank*)user;
    const char* so[2] = {(const char*)send_l, (const char*)send_r};
    char* ri[2] = {(char*)recv_l, (char*)recv_r};
    size_t sn[2] = {bsl, bsr}, rn[2] = {brl, brr};
    const int fd[2] = {R.left_fd, R.right_fd};
    while (sn[0] || sn[1] || rn[0] || rn[1]) {
        pollfd pf[2];
        for (int k = 0; k < 2; ++k) {
            pf[k].fd = fd[k];
            pf[k].events = (short)((sn[k] ? POLLOUT : 0) | (rn[k] ? POLLIN : 0));
            pf[k].revents = 0;
        }
        if (poll(pf, 2, 600000) <= 0) return 1;   // 10 minutes without progress: a dead peer
        for (int k = 0; k < 2; ++k) {
            if (pf[k].revents & (POLLERR | POLLNVAL)) return 1;
            if (sn[k] && (pf[k].revents & POLLOUT)) {
                const ssize_t w = send(fd[k], so[k], sn[k], MSG_DONTWAIT | MSG_NOSIGNAL);
                if (w < 0 && errno != EAGAIN && errno != EINTR) return 1;
                if (w > 0) { so[k] += w; sn[k] -= (size_t)w; }
            }
            if (rn[k] && (pf[k].revents & (POLLIN | POLLHUP))) {
                const ssize_t r = recv(fd[k], ri[k], rn[k], MSG_DONTWAIT);
                if (r == 0) return 1;
                if (r < 0 && errno != EAGAIN && errno != EINTR) return 1;
                if (r > 0) { ri[k] += r; rn[k] -= (size_t)r; }
            }
        }
    }
    return 0;
}

// fork the ranks 1..N-1 (before anything touches the GPU); returns this process's rank
static int spawn_ranks(SlabRank& R, int n, bool host)
{
    R.nranks = n;
    std::vector<int> link(2 * n, -1);   // ring link k: rank k (right side) <-> rank k+1 (left side)
    if (host)
        for (int k = 0; k < n; ++k)
            if (socketpair(AF_UNIX, SOCK_STREAM, 0, &link[2 * k]) != 0) return -1;
    std::vector<int> pipes(2 * n, -1);
    if (!host)
        for (int r = 1; r < n; ++r)
            if (pipe(&pipes[2 * r]) != 0) return -1;
    std::fflush(nullptr);
    if (n > kMaxRanks) return -1;
    struct sigaction sa {};
    sa.sa_handler = on_sigchld;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_RESTART | SA_NOCLDSTOP;
    if (sigaction(SIGCHLD, &sa, nullptr) != 0) return -1;
    // children are registered with SIGCHLD blocked, so the handler never sees a pid it cannot match
    sigset_t blk, old;
    sigemptyset(&blk);
    sigaddset(&blk, SIGCHLD);
    sigprocmask(SIG_BLOCK, &blk, &old);
    const pid_t parent = getpid();
    int me = 0;
    for (int r = 1; r < n; ++r) {
        const pid_t pid = fork();
        if (pid < 0) { sigprocmask(SIG_SETMASK, &old, nullptr); kill_children(); return -1; }
        if (pid == 0) {
            me = r;
            R.children.clear();
            g_nchildren = 0;
            signal(SIGCHLD, SIG_DFL);
            prctl(PR_SET_PDEATHSIG, SIGKILL);   // rank 0 gone: this rank goes too
            if (getppid() != parent) _exit(1);  // (it died before the line above)
            break;
        }
        R.children.push_back(pid);
        g_child_pid[g_nchildren] = pid;
        g_child_done[g_nchildren] = 0;
        g_nchildren = g_nchildren + 1;
    }
    sigprocmask(SIG_SETMASK, &old, nullptr);
    R.rank = me;
    if (host) {
        R.right_fd = link[2 * me];
        R.left_fd = link[2 * ((me + n - 1) % n) + 1];
        for (int k = 0; k < 2 * n; ++k)
            if (link[k] != R.right_fd && link[k] != R.left_fd) close(link[k]);
    } else {
        for (int r = 1; r < n; ++r) {
            if (me == 0) {
                R.uid_out.push_back(pipes[2 * r + 1]);
                close(pipes[2 * r]);
            } else if (r == me) {
                R.uid_fd = pipes[2 * r];
                close(pipes[2 * r + 1]);
            } else {
                close(pipes[2 * r]);
                close(pipes[2 * r + 1]);
            }
        }
    }
    return me;
}

int main(int argc, char** argv)
{
    std::string data = "sample.data", grid = "sample.grid", prof = "sample%03d.prof",
                vtk = "sample%03d.vtk", logname = "sample.log";
    int device = 0;
    if (argc > 1) data = argv[1];
    if (argc > 2) grid = argv[2];
    if (argc > 3) prof = argv[3];
    if (argc > 4) vtk = argv[4];
    if (argc > 5) logname = argv[5];
    // argv[6] is the reference's OpenMP thread count: accepted and ignored
    if (argc > 7) device = std::atoi(argv[7]);
    SlabRank R;
    const int nslabs = std::getenv("MPH_SLABS") ? std::atoi(std::getenv("MPH_SLABS")) : 1;
    const bool host_transport = std::getenv("MPH_SLAB_TRANSPORT") && std::strcmp(std::getenv("MPH_SLAB_TRANSPORT"), "host") == 0;
    if (nslabs > 1 && spawn_ranks(R, nslabs, host_transport) < 0) {
        std::fprintf(stderr, "error: could not start %d slab ranks\n", nslabs);
        return 1;
    }
    const bool root = R.rank == 0;
    g_quiet = !root;
    if (root) g_log = std::fopen(logname.c_str(), "w");
    {
        time_t t = time(nullptr);
        logf("start reading files at %s\n", ctime(&t));
    }
    MphConfig cfg;
    mph_config_default(&cfg, 2, MPH_MODULE_BAR);
    if (const char* d = std::getenv("MPH_DIM")) cfg.dim = std::atoi(d);
    if (const char* m = std::getenv("MPH_MODULE")) {
        // the module #define of main.cpp:54-59 by name (or MphModule number)
        static const char* names[] = {"bar", "dam", "turek_hron", "rolling1", "hydroelastic", "none"};
        cfg.module = std::atoi(m);
        for (int k = 0; k < 6; ++k)
            if (std::strcmp(m, names[k]) == 0) cfg.module = k;
    }
    // the `Rolling` wall-motion #define of main.cpp:58 (calculateWall 2974-3030)
    if (const char* w = std::getenv("MPH_WALL_MOTION"))
        cfg.wall_motion = std::strcmp(w, "rolling") == 0 ? MPH_WALL_ROLLING : std::atoi(w);
    int rc = mph_read_data_file(data.c_str(), &cfg);
    if (rc) die(nullptr, rc, "reading the data file");
    int n = 0;
    rc = mph_read_grid_header(grid.c_str(), &cfg, &n);
    if (rc) die(nullptr, rc, "reading the grid header");
    std::vector<int> prop(n);
    std::vector<double> pos(3 * (size_t)n), pos0(3 * (size_t)n), vel(3 * (size_t)n);
    rc = mph_read_grid_particles(grid.c_str(), n, prop.data(), pos.data(), pos0.data(), vel.data());
    if (rc) die(nullptr, rc, "reading the grid particles");
    int counts[3] = {0, 0, 0};
    for (int t : prop) counts[t < 2 ? 0 : (t < 4 ? 1 : 2)]++;
    if (root)
        std::printf("Fluid Particles: %d\nStructure Particles: %d\nWall Particles: %d\n", counts[0], counts[1], counts[2]);
    {
        time_t t = time(nullptr);
        logf("start initialization at %s\n", ctime(&t));
    }
    MphCtx* ctx = nullptr;
    if (nslabs > 1) {
        // one slab rank: every rank reads the same files and keeps the particles of its slab
        MphSlabOptions o{};
        o.rank = R.rank;
        o.nranks = nslabs;
        o.axis = std::getenv("MPH_SLAB_AXIS") ? std::atoi(std::getenv("MPH_SLAB_AXIS")) : (cfg.dim == 3 ? 2 : 0);
        char uid[128] = {0};
        if (host_transport) {
            o.host_fn = socket_exchange;
            o.host_user = &R;
        } else {
            if (root) {
                rc = mph_dist_unique_id(uid);
                if (rc) die(nullptr, rc, "mph_dist_unique_id");
                for (int fd : R.uid_out)
                    if (!write_all(fd, uid, sizeof(uid))) die(nullptr, MPH_ERR_TRANSPORT, "handing out the RCCL id");
            } else if (!read_all(R.uid_fd, uid, sizeof(uid))) {
                die(nullptr, MPH_ERR_TRANSPORT, "receiving the RCCL id");
            }
            o.unique_id128 = uid;
        }
        if (!(std::getenv("MPH_SLAB_SHARE_DEVICE") && std::atoi(std::getenv("MPH_SLAB_SHARE_DEVICE")))) {
            int ndev = 0;
            if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) device = (device + R.rank) % ndev;
        }
        rc = mph_create_slab(&ctx, &cfg, n, prop.data(), pos.data(), pos0.data(), vel.data(), device, &o);
        if (rc) die(ctx, rc, "mph_create_slab");
    } else {
        rc = mph_create(&ctx, &cfg, n, prop.data(), pos.data(), pos0.data(), vel.data(), device);
        if (rc) die(ctx, rc, "mph_create");
    }
    double sc[36];
    mph_get_scalars(ctx, sc);
    logf("N0a = %e\nN0p = %e\n", sc[0], sc[1]);
    rc = mph_write_vtk(ctx, "output.vtk");
    if (rc) die(ctx, rc, "writing output.vtk");
    {
        time_t t = time(nullptr);
        logf("start main roop at %s\n", ctime(&t));
    }
    // the reference's timing buckets (main.cpp:695-700) from HIP events, opt-in (single GPU,
    // MPH_PHASE_TIMING=1): with them on, mph_step launches every step's kernels directly instead of
    // replaying the captured graphs (HIP cannot time events inside a graph) and waits for the
    // events after every batch of up to 8 steps
    const bool phases = nslabs == 1 && std::getenv("MPH_PHASE_TIMING") && std::atoi(std::getenv("MPH_PHASE_TIMING")) == 1;
    if (phases) {
        rc = mph_phase_timing(ctx, 1);
        if (rc) die(ctx, rc, "mph_phase_timing");
    }
    const auto loop_t0 = std::chrono::steady_clock::now();
    double time_now = cfg.time;
    const double dt = cfg.dt;
    int istep = (int)(time_now / dt);
    double out_next = 0.0, vtk_next = 0.0;
    const bool vtu = vtk.size() > 4 && vtk.compare(vtk.size() - 4, 4, ".vtu") == 0;
    long long steps_run = 0;
    double loop_s = 0.0;
    char name[1024];
    while (time_now < cfg.end_time + 1.0e-5 * dt) {
        if (time_now + 1.0e-5 * dt >= out_next) {
            std::snprintf(name, sizeof(name), prof.c_str(), istep);
            roctxRangePushA("write_prof");
            rc = mph_write_prof(ctx, name);
            roctxRangePop();
            if (rc) die(ctx, rc, "writing a .prof file");
            logf("@ Prof Output Time : %e\n", time_now);
            out_next += cfg.output_interval;
        }
        // run until the next step that produces output (same Time additions as the reference)
        int k = 0;
        double t = time_now;
        bool vtk_after = false;
        while (t < cfg.end_time + 1.0e-5 * dt) {
            ++k;
            if (t + 1.0e-5 * dt >= vtk_next) { vtk_after = true; break; }
            t += dt;
            if (t + 1.0e-5 * dt >= out_next || !(t < cfg.end_time + 1.0e-5 * dt)) break;
        }
        const auto t0 = std::chrono::steady_clock::now();
        roctxRangePushA("mph_step");
        rc = mph_step(ctx, k);
        if (rc) die(ctx, rc, "mph_step");
        mph_synchronize(ctx);
        roctxRangePop();
        // fault injection for the failure-propagation test (tests/test_gpu_driver.py): this rank
        // fails after its first batch
        if (const char* f = std::getenv("MPH_FAIL_RANK"))
            if (nslabs > 1 && std::atoi(f) == R.rank) die(ctx, MPH_ERR_ARG, "MPH_FAIL_RANK fault injection");
        loop_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        steps_run += k;
        for (int s = 0; s < k; ++s) {
            if (vtk_after && s == k - 1) {
                // main.cpp:672-673: the virial diagnostic runs before every VTK write
                roctxRangePushA("virial");
                rc = mph_compute_virial(ctx);
                roctxRangePop();
                if (rc) die(ctx, rc, "mph_compute_virial");
                std::snprintf(name, sizeof(name), vtk.c_str(), istep);
                // formatted and written by a background thread while the next steps run
                rc = vtu ? mph_write_vtu(ctx, name) : mph_write_vtk_async(ctx, name);
                if (rc) die(ctx, rc, "writing a .vtk file");
                logf("@ Vtk Output Time : %e\n", time_now);
                vtk_next += cfg.vtk_output_interval;
            }
            time_now += dt;
            istep++;
        }
    }
    {
        const double total_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - loop_t0).count();
        time_t t = time(nullptr);
        logf("end main roop at %s\n", ctime(&t));
        if (phases) {
            // main.cpp:695-700, in GPU seconds from HIP events; "other" is the rest of the loop's
            // wall time (file output, host work, launch gaps)
            double ph[3] = {0.0, 0.0, 0.0};
            mph_phase_times(ctx, ph);
            const double nb = ph[0] * 1e-3, ex = ph[1] * 1e-3, vi = ph[2] * 1e-3;
            const double other = total_s - nb - ex - vi;
            logf("neighbor search:         %lf [GPU sec]\n", nb);
            logf("explicit calculation:    %lf [GPU sec]\n", ex);
            logf("virial calculation:      %lf [GPU sec]\n", vi);
            logf("other calculation:       %lf [sec]\n", other);
            logf("total:                   %lf [sec]\n", nb + ex + vi + other);
            logf("total (check):           %lf [sec]\n", total_s);
        }
        logf("step loop (wall):        %lf [sec] for %lld steps\n", loop_s, steps_run);
        if (loop_s > 0)
            logf("throughput:              %e [particle-steps/sec]\n", (double)n * steps_run / loop_s);
    }
    rc = mph_output_wait(ctx);
    if (rc) die(ctx, rc, "writing a .vtk file");
    mph_destroy(ctx);
    if (g_log) std::fclose(g_log);
    // rank 0 waits for the other ranks (the SIGCHLD handler reaps them and ends the run if one failed)
    for (;;) {
        bool running = false;
        for (int k = 0; k < g_nchildren; ++k) running = running || g_child_done[k] == 0;
        if (!running) break;
        usleep(1000);
    }
    return 0;
}
