/*
 * mph_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, gcc) of the reference hot path, Ryo1011gd/ParticleMethod_FSI
 * src/main.cpp.  It is the checker for the HIP product path and the `port` CPU baseline of
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * It is pinned against the reference itself: tests/test_oracle.py compares it with golden
 * vectors produced by the compiled reference (oracle/_ref, tests/golden/make_golden.py) and
 * with the live reference library when present -- bit for bit, because it reproduces the
 * reference's loop orders (bitonic cell sort, cell-scan neighbour order, per-kernel sums).
 */
#ifndef MPH_ORACLE_H_INCLUDED
#define MPH_ORACLE_H_INCLUDED

#include "../include/mph_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OrcState OrcState;

OrcState* orc_create(const MphConfig* cfg, int n, const int* property, const double* pos,
                     const double* pos0, const double* vel);
void orc_destroy(OrcState* s);
/* main.cpp:564-570 */
void orc_init(OrcState* s);
/* nsteps x (main.cpp:597-665, Time += Dt) */
void orc_step(OrcState* s, int nsteps);
/* one stage by the reference function name (per-kernel snapshots); 0 ok, -1 unknown */
int orc_call(OrcState* s, const char* name);
/* copy a field out (same names as ref_harness ref_get); returns element count or -1 */
int orc_get(OrcState* s, const char* name, void* out);
int orc_neighbors(OrcState* s, int i, int* out);
int orc_scalars(OrcState* s, double* out36);
double orc_time(OrcState* s);
int orc_count(OrcState* s);
void orc_set_threads(int nthreads);

#ifdef __cplusplus
}
#endif
#endif
