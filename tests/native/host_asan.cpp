// Host-layer sanitizer driver (ASan + UBSan on the CPU code of libmph_gpu.so: readers, writers,
// derived constants, elastic-solid initialisation).  Built and run by tests/test_native_asan.py.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/mph_gpu.h"

int main(int argc, char** argv)
{
    if (argc < 5) return 2;
    MphConfig cfg;
    if (mph_config_default(&cfg, std::atoi(argv[3]), std::atoi(argv[4]))) return 3;
    if (mph_read_data_file(argv[1], &cfg)) return 4;
    int n = 0;
    if (mph_read_grid_header(argv[2], &cfg, &n)) return 5;
    std::vector<int> prop(n), isnc(n);
    std::vector<double> pos(3 * n), pos0(3 * n), vel(3 * n), N(9 * n), ll(n), lm(n), sc(36);
    if (mph_read_grid_particles(argv[2], n, prop.data(), pos.data(), pos0.data(), vel.data())) return 6;
    if (mph_derive_scalars(&cfg, sc.data())) return 7;
    if (mph_structure_init(&cfg, n, prop.data(), pos0.data(), isnc.data(), N.data(), ll.data(), lm.data())) return 8;
    long sum = 0;
    for (int v : isnc) sum += v;
    std::vector<double> z3(3 * n, 0.0), z9(9 * n, 0.0);
    if (argc > 5) {
        if (mph_write_vtk_arrays(argv[5], n, prop.data(), pos.data(), pos0.data(), vel.data(), z3.data(), z3.data(),
                                 z9.data(), z9.data(), isnc.data(), isnc.data())) return 9;
        if (mph_write_prof_arrays(argv[5], &cfg, 0.0, n, prop.data(), pos.data(), pos0.data(), vel.data())) return 10;
    }
    std::printf("n=%d isnc_sum=%ld N0a=%.17g\n", n, sum, sc[0]);
    return 0;
}
