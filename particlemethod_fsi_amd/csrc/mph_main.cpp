// mph_main.cpp -- `mph_explicit`: drop-in replacement of the reference executable.
//
// Same command line as main.cpp:494-508:
//     mph_explicit <data> <grid> <prof pattern> <vtk pattern> <log> [nthreads] [device]
// Same driver semantics as main.cpp:528-700: read files, initialise, write output.vtk, then
// loop while Time < EndTime + 1e-5*Dt writing the .prof before a step (583-589) and the .vtk
// after a step (672-683).  Differences: the physics runs on one MI355X through libmph_gpu.so;
// the .prof holds the current state (the OpenACC build writes stale host arrays);
// the timing report is wall time of the step loop, not clock() CPU time.  A <vtk pattern> ending
// in ".vtu" writes binary VTK XML files instead (mph_write_vtu).
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "../../include/mph_gpu.h"

static FILE* g_log = nullptr;

static void logf(const char* fmt, ...)
{
    va_list a, b;
    va_start(a, fmt);
    va_copy(b, a);
    if (g_log) vfprintf(g_log, fmt, a);
    vfprintf(stderr, fmt, b);
    va_end(a);
    va_end(b);
    if (g_log) fflush(g_log);
}

static void die(MphCtx* c, int rc, const char* what)
{
    logf("error: %s failed (%d): %s\n", what, rc, c ? mph_last_error(c) : "");
    std::exit(1);
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
    g_log = std::fopen(logname.c_str(), "w");
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
    std::printf("Fluid Particles: %d\nStructure Particles: %d\nWall Particles: %d\n", counts[0], counts[1], counts[2]);
    {
        time_t t = time(nullptr);
        logf("start initialization at %s\n", ctime(&t));
    }
    MphCtx* ctx = nullptr;
    rc = mph_create(&ctx, &cfg, n, prop.data(), pos.data(), pos0.data(), vel.data(), device);
    if (rc) die(ctx, rc, "mph_create");
    double sc[36];
    mph_get_scalars(ctx, sc);
    logf("N0a = %e\nN0p = %e\n", sc[0], sc[1]);
    rc = mph_write_vtk(ctx, "output.vtk");
    if (rc) die(ctx, rc, "writing output.vtk");
    {
        time_t t = time(nullptr);
        logf("start main roop at %s\n", ctime(&t));
    }
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
            rc = mph_write_prof(ctx, name);
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
        rc = mph_step(ctx, k);
        if (rc) die(ctx, rc, "mph_step");
        mph_synchronize(ctx);
        loop_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        steps_run += k;
        for (int s = 0; s < k; ++s) {
            if (vtk_after && s == k - 1) {
                // main.cpp:672-673: the virial diagnostic runs before every VTK write
                rc = mph_compute_virial(ctx);
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
        time_t t = time(nullptr);
        logf("end main roop at %s\n", ctime(&t));
        logf("step loop (wall):        %lf [sec] for %lld steps\n", loop_s, steps_run);
        if (loop_s > 0)
            logf("throughput:              %e [particle-steps/sec]\n", (double)n * steps_run / loop_s);
    }
    rc = mph_output_wait(ctx);
    if (rc) die(ctx, rc, "writing a .vtk file");
    mph_destroy(ctx);
    if (g_log) std::fclose(g_log);
    return 0;
}
