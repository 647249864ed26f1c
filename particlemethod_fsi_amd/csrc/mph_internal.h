// mph_internal.h -- internal declarations shared by the host layer, the context and the kernels.
#pragma once

#include <string>
#include <vector>

#include "mph_params.h"

namespace mph {

// Fixed Lagrangian neighbourhood of the elastic solid, built once on the host
// (calculateInitialNeighbor main.cpp:1497-1658, Lamesconstant 2526-2540, Normalizer 2544-2653).
struct StructureInit {
    std::vector<int> orig;          // structure slot -> original particle index (file order)
    std::vector<int> count;         // InitialStructureNeighborCount per slot
    std::vector<int> offset, nbr;   // CSR of neighbour slots (ascending)
    std::vector<int> in_offset, in_nbr;      // transpose: who lists me (senders of the scatter)
    std::vector<double> pair_out;            // per pair {x0_ij[3], weight(x0_ij)} (host: sum w x0)
    std::vector<double> normalizer;          // [ns][3][3]
    std::vector<double> lame_l, lame_m;
};

void derive_constants(const MphConfig& c, HostDerived& h);
void fill_scalars(const HostDerived& h, const MphConfig& c, double* out36);
// z-slab cell order (DevParams.perm 3 or 4) from the particle positions
int choose_cell_order(const HostDerived& h, int n, const double* pos, double rc);
int choose_grid_origin(const HostDerived& h, int n, const double* pos, int d, int gc, int m);
int choose_grid(const HostDerived& h, int dim, double rc, int sa, int gc[3], double ginv[3], std::string& err,
                int perm = 0);
void make_dev_params(const MphConfig& c, const HostDerived& h, int n, int n_struct, DevParams& P);
// lists = false: only the slots (orig), zero counts and the Lame constants (the device builds the
// lists and normalizers, launch_struct_init)
int build_structure(const MphConfig& c, const HostDerived& h, int n, const int* prop,
                    const double* pos0, StructureInit& S, std::string& err, bool lists = true);

}  // namespace mph
