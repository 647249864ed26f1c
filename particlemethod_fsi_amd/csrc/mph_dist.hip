// mph_dist.hip -- multi-GPU slab decomposition entry points (one process per GPU, RCCL).
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/mph_gpu.h"

extern "C" {

int mph_dist_unique_id(char* out128)
{
    if (!out128) return MPH_ERR_ARG;
    std::memset(out128, 0, 128);
    return MPH_ERR_UNSUPPORTED;
}

int mph_create_dist(MphCtx** ctx, const MphConfig* cfg, int n, const int* property, const double* pos,
                    const double* pos0, const double* vel, int device, int rank, int nranks,
                    const char* unique_id128, int axis)
{
    (void)cfg; (void)n; (void)property; (void)pos; (void)pos0; (void)vel; (void)device;
    (void)rank; (void)nranks; (void)unique_id128; (void)axis;
    if (ctx) *ctx = nullptr;
    return MPH_ERR_UNSUPPORTED;
}

int mph_owned_count(const MphCtx* ctx) { return mph_particle_count(ctx); }

}  // extern "C"
