/*
 * mph_oracle.c -- TEST INFRASTRUCTURE ONLY (checker + `port` CPU baseline; never shipped).
 *
 * Clean-room CPU restatement of the reference hot path of Ryo1011gd/ParticleMethod_FSI,
 * src/main.cpp.  Every routine cites the reference lines it restates.  The restatement keeps
 * the reference's evaluation order on purpose (left-to-right products, per-kernel partial sums,
 * bitonic cell sort, cell-scan neighbour order, serial stress-force scatter) and is compiled with
 * -ffp-contract=off, so on the same inputs it reproduces the g++ -O3 build of the reference bit
 * for bit (pinned by tests/test_oracle.py against tests/golden/ and oracle/_ref).
 *
 * Differences from the reference that do not change results:
 *   - the two compile-time switches (TWO_DIMENSIONAL main.cpp:50, case module main.cpp:54-59)
 *     are runtime fields of MphConfig;
 *   - state lives in an OrcState struct instead of file-scope globals;
 *   - the reference's one-past-the-end write CellParticleBegin[CellCounts] (main.cpp:1725 when
 *     the padding key follows the last particle) lands in an allocated spare slot.
 */
#include "mph_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NT MPH_TYPE_COUNT
/* MAXN: the reference's list capacity; MPH_ORACLE_MAXN shrinks the row stride for memory (the
 * D16M fixture build, tools/make_d16m_ncount.py: 128 >= the case's 80; overflow still detected) */
#ifdef MPH_ORACLE_MAXN
#define MAXN MPH_ORACLE_MAXN
#else
#define MAXN MPH_MAX_NEIGHBOR_COUNT
#endif
/* type classes, main.cpp:68-74 */
#define IS_FLUID(t) ((t) >= 0 && (t) < 2)
#define IS_STRUCT(t) ((t) >= 2 && (t) < 4)

typedef double v3[3];
typedef double m33[3][3];

struct OrcState {
    MphConfig c;
    int dim, n;
    /* class ranges, main.cpp:909-929 */
    int fluid_b, fluid_e, struct_b, struct_e, wall_b, wall_e;
    /* derived constants */
    double dx, vol, time, dt, edt;
    double dmin[3], dmax[3], dw[3];
    double ra, rg, rp, rv, max_radius;
    double swa, swg, swp, swv, n0a, n0p, r2g, cofk, cofa[NT];
    double wall_rot[NT][3][3], wall_c[NT][3];
    double cell_w;
    int cell_n[3], cell_total, pow2, pow2_exp;
    /* per particle */
    int *prop;
    v3 *x, *x0, *v, *f, *acc, *gc;
    double *mass, *kappa, *lambda, *mu, *young, *dens_a, *pres_a, *vstrain, *div_p, *pres_p;
    double *lame_l, *lame_m;
    m33 *normalizer, *deform, *strain, *stress;
    m33 *virial;              /* VirialStressAtParticle */
    double *vpres;            /* VirialPressureAtParticle */
    int *ncount, *nlist;     /* [n][MAXN] like main.cpp:877-878 */
    int *sncount, *snlist;   /* InitialStructureNeighbor */
    int *cell_index, *cell_particle, *cell_begin, *cell_end;
};

/* main.cpp:98 */
static inline double orc_mod(double x, double w) { return x - w * floor(x / w); }

/* periodic minimum image used in every pair loop, e.g. main.cpp:1762, 2158 */
static inline double orc_image(const OrcState* s, double a, double b, int d)
{
    return orc_mod(a - b + 0.5 * s->dw[d], s->dw[d]) - 0.5 * s->dw[d];
}

/* kernel functions main.cpp:267-368; h^dim with dim from TWO_DIMENSIONAL */
static inline double hd(const OrcState* s, double h) { return s->dim == 2 ? (h * h) : (h * h * h); }
static double k_wa(const OrcState* s, double r, double h)
{
    return 1.0 / s->swa * 1.0 / hd(s, h) * (r / h) * (1.0 - (r / h)) * (1.0 - (r / h));
}
static double k_dwa(const OrcState* s, double r, double h)
{
    return 1.0 / s->swa * 1.0 / hd(s, h) * (1.0 - (r / h)) * (1.0 - 3.0 * (r / h)) * (1.0 / h);
}
static double k_w2(double sw, double hdv, double r, double h)   /* wg, wp, wv */
{
    return 1.0 / sw * 1.0 / hdv * ((1.0 - r / h) * (1.0 - r / h));
}
static double k_dw2(double sw, double hdv, double r, double h)  /* dwgdr, dwpdr, dwvdr */
{
    return 1.0 / sw * 1.0 / hdv * (-2.0 / h * (1.0 - r / h));
}
static double k_wg(const OrcState* s, double r, double h) { return k_w2(s->swg, hd(s, h), r, h); }
static double k_dwg(const OrcState* s, double r, double h) { return k_dw2(s->swg, hd(s, h), r, h); }
static double k_wp(const OrcState* s, double r, double h) { return k_w2(s->swp, hd(s, h), r, h); }
static double k_dwp(const OrcState* s, double r, double h) { return k_dw2(s->swp, hd(s, h), r, h); }
static double k_dwv(const OrcState* s, double r, double h) { return k_dw2(s->swv, hd(s, h), r, h); }
/* weight(), main.cpp:268-295: norm over 2 or 3 components, normalised with Swp */
static double k_weight(const OrcState* s, const double* rij, double radius)
{
    double r2 = 0.0;
    for (int d = 0; d < (s->dim == 2 ? 2 : 3); ++d) r2 += rij[d] * rij[d];
    double r = sqrt(r2);
    double q = r / radius;
    if (s->dim == 2) return (1.0 / s->swp) * (1.0 / (radius * radius)) * ((1.0 - q) * (1.0 - q));
    return (1.0 / s->swp) * (1.0 / (radius * radius * radius)) * ((1.0 - q) * (1.0 - q));
}

/* CellId macro, main.cpp:122-126 */
static inline int orc_cell_id(const OrcState* s, int cx, int cy, int cz)
{
    const int* C = s->cell_n;
    if (s->dim == 2) return ((cx % C[0] + C[0]) % C[0]) * C[1] + ((cy % C[1] + C[1]) % C[1]);
    return ((cx % C[0] + C[0]) % C[0]) * C[1] * C[2] + ((cy % C[1] + C[1]) % C[1]) * C[2]
           + ((cz % C[2] + C[2]) % C[2]);
}

static inline int orc_axis_cell(const OrcState* s, double x, int d)
{
    return ((int)floor((x - s->dmin[d]) / s->cell_w)) % s->cell_n[d];
}

/* ---------------------------------------------------------------- initialisation ---------- */

/* initializeWeight, main.cpp:1191-1309 */
static void orc_init_weight(OrcState* s)
{
    const double dx = s->dx;
    s->ra = s->c.radius_ratio_a * dx;
    s->rg = s->c.radius_ratio_a * dx;  /* RadiusRatioG = RadiusRatioA, main.cpp:1193 */
    s->rp = s->c.radius_ratio_p * dx;
    s->rv = s->c.radius_ratio_v * dx;
    if (s->dim == 2) {
        s->swa = 1.0 / 2.0 * 2.0 / 15.0 * M_PI / dx / dx;
        s->swg = 1.0 / 2.0 * 1.0 / 3.0 * M_PI / dx / dx;
        s->swp = 1.0 / 2.0 * 1.0 / 3.0 * M_PI / dx / dx;
        s->swv = 1.0 / 2.0 * 1.0 / 3.0 * M_PI / dx / dx;
        s->r2g = 1.0 / 2.0 * 1.0 / 30.0 * M_PI * s->rg * s->rg / dx / dx / s->swg;
    } else {
        s->swa = 1.0 / 3.0 * 1.0 / 5.0 * M_PI / dx / dx / dx;
        s->swg = 1.0 / 3.0 * 2.0 / 5.0 * M_PI / dx / dx / dx;
        s->swp = 1.0 / 3.0 * 2.0 / 5.0 * M_PI / dx / dx / dx;
        s->swv = 1.0 / 3.0 * 2.0 / 5.0 * M_PI / dx / dx / dx;
        s->r2g = 1.0 / 3.0 * 4.0 / 105.0 * M_PI * s->rg * s->rg / dx / dx / dx / s->swg;
    }
    /* lattice sums N0a (main.cpp:1216-1259) and N0p (1261-1304) */
    for (int which = 0; which < 2; ++which) {
        const double R = which == 0 ? s->ra : s->rp;
        const int range = (int)(R / dx + 3.0);
        double sum = 0.0;
        for (int ix = -range; ix <= range; ++ix)
            for (int iy = -range; iy <= range; ++iy)
                for (int iz = (s->dim == 2 ? 0 : -range); iz <= (s->dim == 2 ? 0 : range); ++iz) {
                    if (ix == 0 && iy == 0 && iz == 0) continue;
                    const double x = dx * ((double)ix), y = dx * ((double)iy), z = dx * ((double)iz);
                    const double r2 = s->dim == 2 ? x * x + y * y : x * x + y * y + z * z;
                    if (r2 <= R * R) {
                        const double r = sqrt(r2);
                        sum += which == 0 ? k_wa(s, r, R) : k_wp(s, r, R);
                    }
                }
        if (which == 0) s->n0a = sum; else s->n0p = sum;
    }
}

/* initializeFluid, main.cpp:1312-1367 */
static void orc_init_fluid(OrcState* s)
{
    for (int i = 0; i < s->n; ++i) {
        const int t = s->prop[i];
        s->mass[i] = s->c.density[t] * s->vol;
        s->kappa[i] = s->c.bulk_modulus[t];
        s->lambda[i] = s->c.bulk_viscosity[t];
        s->mu[i] = s->c.shear_viscosity[t];
        s->young[i] = s->c.young_modulus[t];
    }
    double integN, integX;
    if (s->dim == 2) { s->cofk = 0.350778153; integN = 0.024679383; integX = 0.226126699; }
    else { s->cofk = 0.326976006; integN = 0.021425779; integX = 0.233977488; }
    for (int t = 0; t < NT; ++t)
        s->cofa[t] = s->c.surface_tension[t] / ((s->rg / s->dx) * (integN + s->cofk * s->cofk * integX));
}

/* initializeWall, main.cpp:1371-1410 (note theta is the SQUARED norm of omega, as there) */
static void orc_init_wall(OrcState* s)
{
    memset(s->wall_rot, 0, sizeof s->wall_rot);
    for (int t = 4; t < 6; ++t) {
        const double* w = s->c.wall_omega[t];
        double nrm[3] = {0.0, 0.0, 0.0}, q[4];
        double theta = fabs(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        if (theta != 0.0)
            for (int d = 0; d < 3; ++d) nrm[d] = w[d] / theta;
        q[0] = nrm[0] * sin(theta * s->dt / 2.0);
        q[1] = nrm[1] * sin(theta * s->dt / 2.0);
        q[2] = nrm[2] * sin(theta * s->dt / 2.0);
        q[3] = cos(theta * s->dt / 2.0);
        double (*R)[3] = s->wall_rot[t];
        R[0][0] = q[0] * q[0] - q[1] * q[1] - q[2] * q[2] + q[3] * q[3];
        R[0][1] = 2.0 * (q[0] * q[1] - q[2] * q[3]);
        R[0][2] = 2.0 * (q[0] * q[2] + q[1] * q[3]);
        R[1][0] = 2.0 * (q[0] * q[1] + q[2] * q[3]);
        R[1][1] = -q[0] * q[0] + q[1] * q[1] - q[2] * q[2] + q[3] * q[3];
        R[1][2] = 2.0 * (q[1] * q[2] - q[0] * q[3]);
        R[2][0] = 2.0 * (q[0] * q[2] - q[1] * q[3]);
        R[2][1] = 2.0 * (q[1] * q[2] + q[0] * q[3]);
        R[2][2] = -q[0] * q[0] - q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    }
}

/* initializeDomain, main.cpp:1412-1469 */
static void orc_init_domain(OrcState* s)
{
    s->cell_w = s->dx;
    double cc[3];
    cc[0] = round((s->dmax[0] - s->dmin[0]) / s->cell_w);
    cc[1] = round((s->dmax[1] - s->dmin[1]) / s->cell_w);
    cc[2] = s->dim == 2 ? 1 : round((s->dmax[2] - s->dmin[2]) / s->cell_w);
    for (int d = 0; d < 3; ++d) s->cell_n[d] = (int)cc[d];
    s->cell_total = (int)(cc[0] * cc[1] * cc[2]);
    if (cc[0] != (double)s->cell_n[0] || cc[1] != (double)s->cell_n[1] || cc[2] != (double)s->cell_n[2])
        for (int d = 0; d < 3; ++d) s->dmax[d] = s->dmin[d] + s->cell_w * (double)s->cell_n[d];
    for (int d = 0; d < 3; ++d) s->dw[d] = s->dmax[d] - s->dmin[d];
    s->pow2_exp = 0;
    while ((s->n >> s->pow2_exp) != 0) ++s->pow2_exp;
    s->pow2 = 1 << s->pow2_exp;
    s->max_radius = 0.0;
    const double radii[4] = {s->ra, s->rg, s->rp, s->rv};
    for (int k = 0; k < 4; ++k) s->max_radius = radii[k] > s->max_radius ? radii[k] : s->max_radius;
}

/* ---------------------------------------------------------------- neighbour search --------- */

/* cell keys + bitonic sort + cell ranges: main.cpp:1666-1728 (also 1501-1563 on x0) */
static void orc_build_cells(OrcState* s, v3* pos)
{
    const int P = s->pow2, n = s->n;
    #pragma omp parallel for
    for (int i = 0; i < P; ++i) {
        if (i < n) {
            const int cx = orc_axis_cell(s, pos[i][0], 0);
            const int cy = orc_axis_cell(s, pos[i][1], 1);
            const int cz = orc_axis_cell(s, pos[i][2], 2);
            s->cell_index[i] = orc_cell_id(s, cx, cy, cz);
            s->cell_particle[i] = i;
        } else {
            s->cell_index[i] = s->cell_n[0] * s->cell_n[1] * s->cell_n[2];
            s->cell_particle[i] = n;
        }
    }
    for (int stage = 0; stage < s->pow2_exp; ++stage) {
        for (int sub = 0; sub <= stage; ++sub) {
            const int dist = 1 << (stage - sub);
            #pragma omp parallel for
            for (int i = 0; i < P; ++i) {
                const int up = ((i >> stage) & 2) == 0;
                if ((i & dist) == 0 && ((s->cell_index[i] > s->cell_index[i | dist]) == up)) {
                    int tk = s->cell_index[i], tp = s->cell_particle[i];
                    s->cell_index[i] = s->cell_index[i | dist];
                    s->cell_particle[i] = s->cell_particle[i | dist];
                    s->cell_index[i | dist] = tk;
                    s->cell_particle[i | dist] = tp;
                }
            }
        }
    }
    memset(s->cell_begin, 0, sizeof(int) * (s->cell_total + 1));
    memset(s->cell_end, 0, sizeof(int) * (s->cell_total + 1));
    #pragma omp parallel for
    for (int i = 0; i < n; ++i) {
        if (s->cell_index[i] < s->cell_index[i + 1]) {
            s->cell_end[s->cell_index[i]] = i + 1;
            s->cell_begin[s->cell_index[i + 1]] = i + 1;
        }
    }
}

/* per-particle scan of (2*range+1)^dim cells: main.cpp:1743-1810 (all j) and 1579-1644
 * (structure i, structure j, InitialPosition, 2-D z-component forced to zero)              */
static void orc_scan_neighbors(OrcState* s, v3* pos, int i, int structure_only, int* count, int* list)
{
    const double rc = s->max_radius + (0.1 * s->dx);
    const int range = (int)(ceil((s->max_radius + (0.1 * s->dx)) / s->cell_w));
    const int icx = orc_axis_cell(s, pos[i][0], 0);
    const int icy = orc_axis_cell(s, pos[i][1], 1);
    const int icz = s->dim == 2 ? 0 : orc_axis_cell(s, pos[i][2], 2);
    const int zr = s->dim == 2 ? 0 : range;
    int c = 0;
    for (int jcx = icx - range; jcx <= icx + range; ++jcx)
        for (int jcy = icy - range; jcy <= icy + range; ++jcy)
            for (int jcz = icz - zr; jcz <= icz + zr; ++jcz) {
                const int jc = orc_cell_id(s, jcx, jcy, jcz);
                for (int k = s->cell_begin[jc]; k < s->cell_end[jc]; ++k) {
                    const int j = s->cell_particle[k];
                    double q[3];
                    if (structure_only) {
                        q[0] = orc_image(s, pos[j][0], pos[i][0], 0);
                        q[1] = orc_image(s, pos[j][1], pos[i][1], 1);
                        q[2] = s->dim == 2 ? 0.0 : orc_image(s, pos[j][2], pos[i][2], 2);
                    } else {
                        for (int d = 0; d < 3; ++d) q[d] = orc_image(s, pos[j][d], pos[i][d], d);
                    }
                    const double q2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2];
                    int ok = q2 <= rc * rc;
                    if (structure_only) ok = ok && IS_STRUCT(s->prop[j]);
                    if (ok) {
                        if (c >= MAXN) c++;
                        else if (i != j) list[c++] = j;
                    }
                }
            }
    *count = c;
}

/* calculateNeighbor, main.cpp:1662-1822 */
static void orc_neighbor(OrcState* s)
{
    orc_build_cells(s, s->x);
    #pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < s->n; ++i) {
        int* row = s->nlist + (size_t)i * MAXN;
        for (int k = 0; k < MAXN; ++k) row[k] = -1;
        orc_scan_neighbors(s, s->x, i, 0, &s->ncount[i], row);
    }
}

/* calculateInitialNeighbor, main.cpp:1497-1658 */
static void orc_initial_neighbor(OrcState* s)
{
    orc_build_cells(s, s->x0);
    #pragma omp parallel for schedule(dynamic, 64)
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        int* row = s->snlist + (size_t)i * MAXN;
        for (int k = 0; k < MAXN; ++k) row[k] = -1;
        orc_scan_neighbors(s, s->x0, i, 1, &s->sncount[i], row);
    }
}

/* ---------------------------------------------------------------- fluid sums --------------- */

static inline void orc_pair(const OrcState* s, int i, int j, double xij[3], double* r2)
{
    for (int d = 0; d < 3; ++d) xij[d] = orc_image(s, s->x[j][d], s->x[i][d], d);
    *r2 = (xij[0] * xij[0] + xij[1] * xij[1] + xij[2] * xij[2]);
}

/* calculateDensityA, main.cpp:2141-2171 */
static void orc_density_a(OrcState* s)
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        if (IS_STRUCT(s->prop[i])) continue;
        double sum = 0.0;
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            const double ratio = s->c.interaction_ratio[s->prop[i]][s->prop[j]];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->ra * s->ra - r2 >= 0) {
                const double r = sqrt(r2);
                sum += ratio * k_wa(s, r, s->ra);
            }
        }
        s->dens_a[i] = sum;
    }
}

/* calculateGravityCenter, main.cpp:2174-2210 */
static void orc_gravity_center(OrcState* s)
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        if (IS_STRUCT(s->prop[i])) continue;
        double sum[3] = {0.0, 0.0, 0.0};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            const double ratio = s->c.interaction_ratio[s->prop[i]][s->prop[j]];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rg * s->rg - r2 >= 0) {
                const double r = sqrt(r2);
                const double w = ratio * k_wg(s, r, s->rg);
                for (int d = 0; d < 3; ++d) sum[d] += xij[d] * w / s->r2g * s->rg;
            }
        }
        for (int d = 0; d < 3; ++d) s->gc[i][d] = sum[d];
    }
}

/* calculatePressureA, main.cpp:2212-2259 */
static void orc_pressure_a(OrcState* s)
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        s->pres_a[i] = s->cofa[s->prop[i]] * (s->dens_a[i] - s->n0a) / s->dx;
        if (s->n0a <= s->dens_a[i]) s->pres_a[i] = 0.0;
    }
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        if (IS_STRUCT(s->prop[i])) continue;
        double force[3] = {0.0, 0.0, 0.0};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            const double rij_ = s->c.interaction_ratio[s->prop[i]][s->prop[j]];
            const double rji_ = s->c.interaction_ratio[s->prop[j]][s->prop[i]];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->ra * s->ra - r2 > 0) {
                const double r = sqrt(r2);
                const double dwij = rij_ * k_dwa(s, r, s->ra);
                const double dwji = rji_ * k_dwa(s, r, s->ra);
                const double e[3] = {xij[0] / r, xij[1] / r, xij[2] / r};
                for (int d = 0; d < 3; ++d)
                    force[d] += (s->pres_a[i] * dwij + s->pres_a[j] * dwji) * e[d] * s->vol;
            }
        }
        for (int d = 0; d < 3; ++d) s->f[i][d] += force[d];
    }
}

/* calculateDiffuseInterface, main.cpp:2261-2312 (a_j uses CofA of type(i), as there) */
static void orc_diffuse_interface(OrcState* s)
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        if (IS_STRUCT(s->prop[i])) continue;
        const double ai = s->cofa[s->prop[i]] * (s->cofk) * (s->cofk);
        double force[3] = {0.0, 0.0, 0.0};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            const double aj = s->cofa[s->prop[i]] * (s->cofk) * (s->cofk);
            const double rij_ = s->c.interaction_ratio[s->prop[i]][s->prop[j]];
            const double rji_ = s->c.interaction_ratio[s->prop[j]][s->prop[i]];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rg * s->rg - r2 > 0) {
                const double r = sqrt(r2);
                const double wij = rij_ * k_wg(s, r, s->rg);
                const double wji = rji_ * k_wg(s, r, s->rg);
                for (int d = 0; d < 3; ++d)
                    force[d] -= (aj * s->gc[j][d] * wji - ai * s->gc[i][d] * wij) / s->r2g * s->rg * (s->vol / s->dx);
                const double dwij = rij_ * k_dwg(s, r, s->rg);
                const double dwji = rji_ * k_dwg(s, r, s->rg);
                const double e[3] = {xij[0] / r, xij[1] / r, xij[2] / r};
                double gr = 0.0;
                for (int d = 0; d < 3; ++d)
                    gr += (aj * s->gc[j][d] * dwji - ai * s->gc[i][d] * dwij) * xij[d];
                for (int d = 0; d < 3; ++d)
                    force[d] -= (gr) * e[d] / s->r2g * s->rg * (s->vol / s->dx);
            }
        }
        for (int d = 0; d < 3; ++d) s->f[i][d] += force[d];
    }
}

/* calculateDensityP, main.cpp:2314-2341 (all particles) */
static void orc_density_p(OrcState* s)
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        double sum = 0.0;
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rp * s->rp - r2 >= 0) {
                const double r = sqrt(r2);
                sum += k_wp(s, r, s->rp);
            }
        }
        s->vstrain[i] = (sum - s->n0p);
    }
}

/* calculateDivergenceP, main.cpp:2343-2379 (all particles) */
static void orc_divergence_p(OrcState* s)
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        double sum = 0.0;
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rp * s->rp - r2 >= 0) {
                const double r = sqrt(r2);
                const double dw = k_dwp(s, r, s->rp);
                const double e[3] = {xij[0] / r, xij[1] / r, xij[2] / r};
                double u[3];
                for (int d = 0; d < 3; ++d) u[d] = s->v[j][d] - s->v[i][d];
                for (int d = 0; d < 3; ++d) sum -= u[d] * e[d] * dw;
            }
        }
        s->div_p[i] = sum;
    }
}

/* calculatePhysicalCoefficients, main.cpp:2099-2137 */
static void orc_coefficients(OrcState* s)
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        const int t = s->prop[i];
        s->mass[i] = s->c.density[t] * s->vol;
        s->kappa[i] = s->c.bulk_modulus[t];
        if (s->vstrain[i] < 0.0) s->kappa[i] = 0.0;
        s->lambda[i] = s->c.bulk_viscosity[t];
        s->mu[i] = s->c.shear_viscosity[t];
        s->young[i] = s->c.young_modulus[t];
    }
}

static void orc_pressure_value(OrcState* s)   /* main.cpp:2384-2392 and 2429-2437 */
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        s->pres_p[i] = -s->lambda[i] * s->div_p[i];
        if (s->vstrain[i] > 0.0) s->pres_p[i] += s->kappa[i] * s->vstrain[i];
    }
}

/* calculatePressureP, main.cpp:2381-2425 */
static void orc_pressure_p(OrcState* s)
{
    orc_pressure_value(s);
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        if (IS_STRUCT(s->prop[i])) continue;
        double force[3] = {0.0, 0.0, 0.0};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rp * s->rp - r2 > 0) {
                const double r = sqrt(r2);
                const double dw = k_dwp(s, r, s->rp);
                const double g[3] = {dw * xij[0] / r, dw * xij[1] / r, dw * xij[2] / r};
                for (int d = 0; d < 3; ++d) force[d] += (s->pres_p[i] + s->pres_p[j]) * g[d] * s->vol;
            }
        }
        for (int d = 0; d < 3; ++d) s->f[i][d] += force[d];
    }
}

/* calculateInterfaceForce, main.cpp:2427-2473 */
static void orc_interface_force(OrcState* s)
{
    orc_pressure_value(s);
    #pragma omp parallel for
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        double force[3] = {0.0, 0.0, 0.0};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            if (IS_STRUCT(s->prop[j])) continue;
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (r2 < s->rp * s->rp) {
                const double r = sqrt(r2);
                const double dw = k_dwp(s, r, s->rp);
                const double g[3] = {dw * xij[0] / r, dw * xij[1] / r, dw * xij[2] / r};
                for (int d = 0; d < 3; ++d) force[d] += (s->pres_p[i] + s->pres_p[j]) * g[d] * s->vol;
            }
        }
        for (int d = 0; d < 3; ++d) s->f[i][d] += force[d];
    }
}

/* calculateViscosityV, main.cpp:2478-2522 */
static void orc_viscosity(OrcState* s)
{
    const double cvis = s->dim == 2 ? 8.0 : 10.0;
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {
        if (IS_STRUCT(s->prop[i])) continue;
        double force[3] = {0.0, 0.0, 0.0};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rv * s->rv - r2 > 0) {
                const double r = sqrt(r2);
                const double dwij = -k_dwv(s, r, s->rv);
                const double e[3] = {xij[0] / r, xij[1] / r, xij[2] / r};
                double u[3];
                for (int d = 0; d < 3; ++d) u[d] = s->v[j][d] - s->v[i][d];
                const double muij = 2.0 * (s->mu[i] * s->mu[j]) / (s->mu[i] + s->mu[j]);
                for (int d = 0; d < 3; ++d)
                    force[d] += cvis * muij * (u[0] * e[0] + u[1] * e[1] + u[2] * e[2]) * e[d] * dwij / r * s->vol;
            }
        }
        for (int d = 0; d < 3; ++d) s->f[i][d] += force[d];
    }
}

/* calculateGravity, main.cpp:2917-2936 */
static void orc_gravity(OrcState* s)
{
    for (int pass = 0; pass < 2; ++pass) {
        const int b = pass == 0 ? s->fluid_b : s->struct_b, e = pass == 0 ? s->fluid_e : s->struct_e;
        for (int i = b; i < e; ++i)
            for (int d = 0; d < 3; ++d) s->f[i][d] += s->mass[i] * s->c.gravity[d];
    }
}

/* calculateAcceleration, main.cpp:2938-2956 */
static void orc_kick(OrcState* s)
{
    for (int pass = 0; pass < 2; ++pass) {
        const int b = pass == 0 ? s->fluid_b : s->struct_b, e = pass == 0 ? s->fluid_e : s->struct_e;
        for (int i = b; i < e; ++i)
            for (int d = 0; d < 3; ++d) s->v[i][d] += s->f[i][d] / s->mass[i] * s->dt;
    }
}

/* calculateConvection, main.cpp:1892-1907 */
static void orc_convection(OrcState* s)
{
    for (int i = s->fluid_b; i < s->fluid_e; ++i) {
        for (int d = 0; d < 3; ++d) s->acc[i][d] += s->f[i][d] / s->mass[i];
        for (int d = 0; d < 3; ++d) s->x[i][d] += s->v[i][d] * s->dt;
    }
}

/* ---------------------------------------------------------------- walls & boundary --------- */

/* calculateWall, main.cpp:2963-3072 (active #else branch 3031-3071) */
static void orc_wall(OrcState* s)
{
    for (int i = s->wall_b; i < s->wall_e; ++i)
        for (int d = 0; d < 3; ++d) s->f[i][d] = 0.0;
    if (s->c.wall_motion == MPH_WALL_ROLLING) {   /* the `Rolling` branch, main.cpp:2974-3029 */
        const double max_angle = (2.0 * M_PI / 180.0), period = 1.646;   /* 2959-2960 */
        const double omega_t = 2.0 * M_PI / period;
        const double theta = max_angle * sin(omega_t * s->time);
        const double dtheta_dt = max_angle * omega_t * cos(omega_t * s->time);
        const double theta_prev = max_angle * sin(omega_t * (s->time - s->dt));
        const double delta_theta = theta - theta_prev;
        const double cosD = cos(delta_theta), sinD = sin(delta_theta);
        const double Rz[3][3] = {{cosD, -sinD, 0.0}, {sinD, cosD, 0.0}, {0.0, 0.0, 1.0}};
        for (int i = s->wall_b; i < s->wall_e; ++i) {
            const int t = s->prop[i];
            const double* C = s->wall_c[t];
            const double r[3] = {s->x[i][0] - C[0], s->x[i][1] - C[1], s->x[i][2] - C[2]};
            double rr[3];
            rr[0] = Rz[0][0] * r[0] + Rz[0][1] * r[1];
            rr[1] = Rz[1][0] * r[0] + Rz[1][1] * r[1];
            rr[2] = r[2];
            const double w[3] = {0.0, 0.0, dtheta_dt};
            s->v[i][0] = w[1] * rr[2] - w[2] * rr[1];
            s->v[i][1] = w[2] * rr[0] - w[0] * rr[2];
            s->v[i][2] = w[0] * rr[1] - w[1] * rr[0];
            s->x[i][0] = rr[0] + C[0];
            s->x[i][1] = rr[1] + C[1];
            s->x[i][2] = rr[2] + C[2];
        }
        for (int t = 4; t < 6; ++t)
            for (int d = 0; d < 3; ++d) s->wall_c[t][d] += s->c.wall_velocity[t][d] * s->dt;
        return;
    }
    for (int i = s->wall_b; i < s->wall_e; ++i) {
        if (!(s->time < 0.2)) continue;
        const int t = s->prop[i];
        const double* C = s->wall_c[t];
        const double* V = s->c.wall_velocity[t];
        const double* w = s->c.wall_omega[t];
        double (*R)[3] = s->wall_rot[t];
        const double r[3] = {s->x[i][0] - C[0], s->x[i][1] - C[1], s->x[i][2] - C[2]};
        double rr[3];
        rr[0] = R[0][0] * r[0] + R[0][1] * r[1] + R[0][2] * r[2];
        rr[1] = R[1][0] * r[0] + R[1][1] * r[1] + R[1][2] * r[2];
        rr[2] = R[2][0] * r[0] + R[2][1] * r[1] + R[2][2] * r[2];
        s->v[i][0] = w[1] * rr[2] - w[2] * rr[1] + V[0];
        s->v[i][1] = w[2] * rr[0] - w[0] * rr[2] + V[1];
        s->v[i][2] = w[0] * rr[1] - w[1] * rr[0] + V[2];
        s->x[i][0] = rr[0] + C[0] + V[0] * s->dt;
        s->x[i][1] = rr[1] + C[1] + V[1] * s->dt;
        s->x[i][2] = rr[2] + C[2] + V[2] * s->dt;
    }
    for (int t = 4; t < 6; ++t)
        for (int d = 0; d < 3; ++d) s->wall_c[t][d] += s->c.wall_velocity[t][d] * s->dt;
}

/* calculatePeriodicBoundary, main.cpp:3322-3333 */
static void orc_periodic(OrcState* s)
{
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i)
        for (int d = 0; d < 3; ++d) s->x[i][d] = orc_mod(s->x[i][d] - s->dmin[d], s->dw[d]) + s->dmin[d];
}

static void orc_reset_force(OrcState* s) { memset(s->f, 0, sizeof(v3) * s->n); }   /* 2085-2096 */
static void orc_reset_accel(OrcState* s) { memset(s->acc, 0, sizeof(v3) * s->n); }  /* 2892-2911 */

/* ---------------------------------------------------------------- elastic solid ------------ */

/* calculateLamesconstant, main.cpp:2526-2540 */
static void orc_lame(OrcState* s)
{
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        const double E = s->c.young_modulus[s->prop[i]], nu = s->c.poisson_ratio[s->prop[i]];
        s->lame_l[i] = (E * nu) / ((1.0 + nu) * (1.0 - 2.0 * nu));
        s->lame_m[i] = E / (2.0 * (1.0 + nu));
    }
}

/* calculateNormalizer, main.cpp:2544-2653 (accumulates 3x3 in both dims: TWO_DIMENSION typo) */
static void orc_normalizer(OrcState* s)
{
    for (int i = s->struct_b; i < s->struct_e; ++i)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) s->normalizer[i][a][b] = 0.0;
    #pragma omp parallel for
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        double (*N)[3] = s->normalizer[i];
        for (int k = 0; k < s->sncount[i]; ++k) {
            const int j = s->snlist[(size_t)i * MAXN + k];
            if (i == j) continue;
            double x0[3] = {0.0};
            for (int d = 0; d < 3; ++d) x0[d] = orc_image(s, s->x0[j][d], s->x0[i][d], d);
            const double w = k_weight(s, x0, s->rp);
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) N[a][b] += w * x0[a] * x0[b];
        }
        if (s->dim == 2) {
            const double a = N[0][0], b = N[0][1], c = N[1][0], d = N[1][1];
            const double det = a * d - b * c;
            if (det != 0.0) {
                const double inv[2][2] = {{d / det, -b / det}, {-c / det, a / det}};
                for (int p = 0; p < 2; ++p)
                    for (int q = 0; q < 2; ++q) N[p][q] = inv[p][q];
            } else {
                for (int p = 0; p < 2; ++p)
                    for (int q = 0; q < 2; ++q) N[p][q] = (p == q) ? 1.0 : 0.0;
            }
        } else {
            const double det = N[0][0] * (N[1][1] * N[2][2] - N[1][2] * N[2][1])
                             - N[0][1] * (N[1][0] * N[2][2] - N[1][2] * N[2][0])
                             + N[0][2] * (N[1][0] * N[2][1] - N[1][1] * N[2][0]);
            if (det != 0.0) {
                double adj[3][3];
                adj[0][0] = N[1][1] * N[2][2] - N[1][2] * N[2][1];
                adj[0][1] = -N[1][0] * N[2][2] + N[1][2] * N[2][0];
                adj[0][2] = N[1][0] * N[2][1] - N[1][1] * N[2][0];
                adj[1][0] = -N[0][1] * N[2][2] + N[0][2] * N[2][1];
                adj[1][1] = N[0][0] * N[2][2] - N[0][2] * N[2][0];
                adj[1][2] = -N[0][0] * N[2][1] + N[0][1] * N[2][0];
                adj[2][0] = N[0][1] * N[1][2] - N[0][2] * N[1][1];
                adj[2][1] = -N[0][0] * N[1][2] + N[0][2] * N[1][0];
                adj[2][2] = N[0][0] * N[1][1] - N[0][1] * N[1][0];
                for (int p = 0; p < 3; ++p)
                    for (int q = 0; q < 3; ++q) N[p][q] = adj[p][q] / det;
            }
        }
    }
}

/* calculateElasticDeformationVector, main.cpp:2673-2754 */
static void orc_deformation(OrcState* s)
{
    const int D = s->dim;
    for (int i = s->struct_b; i < s->struct_e; ++i)
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) s->deform[i][a][b] = 0.0;
    #pragma omp parallel for
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        for (int k = 0; k < s->sncount[i]; ++k) {
            const int j = s->snlist[(size_t)i * MAXN + k];
            if (i == j) continue;
            double ui[3] = {0}, uj[3] = {0}, x0[3] = {0}, xx[3] = {0};
            for (int d = 0; d < D; ++d) {
                ui[d] = orc_image(s, s->x[i][d], s->x0[i][d], d);
                uj[d] = 1.0 * (orc_image(s, s->x[j][d], s->x0[j][d], d));  /* Conversion = I */
                x0[d] = orc_image(s, s->x0[j][d], s->x0[i][d], d);
                xx[d] = x0[d] + (uj[d] - ui[d]);
            }
            const double w = k_weight(s, x0, s->rp);
            for (int a = 0; a < D; ++a)
                for (int b = 0; b < D; ++b) s->deform[i][a][b] += w * xx[a] * x0[b];
        }
    }
    #pragma omp parallel for
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        double tmp[3][3] = {{0.0}};
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) {
                double sum = 0.0;
                for (int k = 0; k < D; ++k) sum += s->deform[i][a][k] * s->normalizer[i][k][b];
                tmp[a][b] = sum;
            }
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) s->deform[i][a][b] = tmp[a][b];
    }
}

/* calculateStress, main.cpp:2756-2809 */
static void orc_stress(OrcState* s)
{
    const int D = s->dim;
    #pragma omp parallel for
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        double e[3][3] = {{0.0}};
        double tr = 0.0;
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) {
                double sum = 0.0;
                for (int k = 0; k < D; ++k) sum += s->deform[i][k][a] * s->deform[i][k][b];
                e[a][b] = 0.5 * (sum - (a == b ? 1.0 : 0.0));
                if (a == b) tr += e[a][b];
            }
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) s->strain[i][a][b] = e[a][b];
        const double mu = s->lame_m[i], la = s->lame_l[i];
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) {
                s->stress[i][a][b] = 2.0 * mu * e[a][b];
                if (a == b) s->stress[i][a][b] += la * tr;
            }
    }
}

/* calculateStressForce, main.cpp:2812-2890: serial, scatter form (no OpenMP pragma there) */
static void orc_stress_force(OrcState* s)
{
    const int D = s->dim;
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        double P[3][3] = {{0.0}};
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) {
                double sum = 0.0;
                for (int k = 0; k < D; ++k)
                    for (int l = 0; l < D; ++l)
                        sum += s->deform[i][a][k] * s->stress[i][k][l] * s->normalizer[i][l][b];
                P[a][b] = sum;
            }
        for (int k = 0; k < s->sncount[i]; ++k) {
            const int j = s->snlist[(size_t)i * MAXN + k];
            if (j == i) continue;
            double x0[3] = {0.0};
            for (int d = 0; d < D; ++d) x0[d] = orc_image(s, s->x0[j][d], s->x0[i][d], d);
            const double w = k_weight(s, x0, s->rp);
            double fv[3] = {0.0};
            for (int a = 0; a < D; ++a) {
                for (int b = 0; b < D; ++b) fv[a] += P[a][b] * x0[b];
                fv[a] *= w;
            }
            const double inv_i = 1.0 / s->c.density[s->prop[i]];
            const double inv_j = 1.0 / s->c.density[s->prop[j]];
            for (int d = 0; d < D; ++d) {
                s->v[i][d] += inv_i * fv[d] * s->edt;
                s->v[j][d] -= inv_j * fv[d] * s->edt;
            }
        }
    }
}

/* updateElasticPosition, main.cpp:1910-2082: module clamp, then the always-compiled
 * `#ifdef Rolling2 ... #else` drift (2070-2079), so free particles drift twice.          */
static void orc_update_elastic(OrcState* s)
{
    const double edt = s->edt;
    for (int i = s->struct_b; i < s->struct_e; ++i) {
        const double* p0 = s->x0[i];
        int clamp = 0, zero_force = 1;
        switch (s->c.module) {
        case MPH_MODULE_BAR: clamp = p0[0] < 0.001; break;
        case MPH_MODULE_DAM: clamp = p0[1] < 0.002; break;
        case MPH_MODULE_TUREK_HRON: clamp = p0[0] < 0.205; zero_force = 0; break;
        case MPH_MODULE_ROLLING1: clamp = p0[1] < 0.003; break;
        case MPH_MODULE_HYDROELASTIC: clamp = p0[0] < 0.01 || p0[0] > 1.99; break;
        default: clamp = -1; break;
        }
        if (clamp == 1) {
            for (int d = 0; d < 3; ++d) { s->x[i][d] = p0[d]; s->v[i][d] = 0.0; }
            if (zero_force)
                for (int d = 0; d < 3; ++d) s->f[i][d] = 0.0;
        } else if (clamp == 0) {
            for (int d = 0; d < 3; ++d) s->v[i][d] += s->acc[i][d] * edt;
            for (int d = 0; d < 3; ++d) s->x[i][d] += s->v[i][d] * edt;
        }
        for (int d = 0; d < 3; ++d) s->v[i][d] += s->acc[i][d] * edt;
        for (int d = 0; d < 3; ++d) s->x[i][d] += s->v[i][d] * edt;
    }
}

/* ---------------------------------------------------------------- driver ------------------- */

/* calculateVirialStressAtParticle, main.cpp:3077-3318: four pair loops, each accumulating its
 * own stress[3][3] per particle and adding it to VirialStressAtParticle, then the pressure. */
static void orc_virial_add(OrcState* s, int i, double st[3][3])
{
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) s->virial[i][a][b] += st[a][b];
}

static void orc_virial(OrcState* s)
{
    const double cvis = s->dim == 2 ? 8.0 : 10.0;
    memset(s->virial, 0, sizeof(m33) * (size_t)s->n);   /* 3083-3093 */
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {   /* pressureP, 3095-3125 */
        double st[3][3] = {{0.0}};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rp * s->rp - r2 > 0) {
                const double r = sqrt(r2);
                const double dwij = k_dwp(s, r, s->rp);
                const double gradw[3] = {dwij * xij[0] / r, dwij * xij[1] / r, dwij * xij[2] / r};
                double fij[3];
                for (int d = 0; d < 3; ++d) fij[d] = (s->pres_p[i]) * gradw[d] * s->vol;
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) st[a][b] += 1.0 * fij[a] * xij[b] / s->vol;
            }
        }
        orc_virial_add(s, i, st);
    }
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {   /* pressureA, 3127-3163 */
        double st[3][3] = {{0.0}};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->ra * s->ra - r2 > 0) {
                const double ratio = s->c.interaction_ratio[s->prop[i]][s->prop[j]];
                const double r = sqrt(r2);
                const double dwij = ratio * k_dwa(s, r, s->ra);
                const double gradw[3] = {dwij * xij[0] / r, dwij * xij[1] / r, dwij * xij[2] / r};
                double fij[3];
                for (int d = 0; d < 3; ++d) fij[d] = (s->pres_a[i]) * gradw[d] * s->vol;
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) st[a][b] += 1.0 * fij[a] * xij[b] / s->vol;
            }
        }
        orc_virial_add(s, i, st);
    }
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {   /* viscosity, 3165-3206 */
        double st[3][3] = {{0.0}};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rv * s->rv - r2 > 0) {
                const double r = sqrt(r2);
                const double dwij = -k_dwv(s, r, s->rv);
                const double e[3] = {xij[0] / r, xij[1] / r, xij[2] / r};
                const double u[3] = {s->v[j][0] - s->v[i][0], s->v[j][1] - s->v[i][1], s->v[j][2] - s->v[i][2]};
                const double muij = 2.0 * (s->mu[i] * s->mu[j]) / (s->mu[i] + s->mu[j]);
                double fij[3];
                for (int d = 0; d < 3; ++d)
                    fij[d] = cvis * muij * (u[0] * e[0] + u[1] * e[1] + u[2] * e[2]) * e[d] * dwij / r * s->vol;
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) st[a][b] += 0.5 * fij[a] * xij[b] / s->vol;
            }
        }
        orc_virial_add(s, i, st);
    }
    #pragma omp parallel for
    for (int i = 0; i < s->n; ++i) {   /* diffuse interface, 3208-3282 */
        double st[3][3] = {{0.0}};
        for (int k = 0; k < s->ncount[i]; ++k) {
            const int j = s->nlist[(size_t)i * MAXN + k];
            double xij[3], r2;
            orc_pair(s, i, j, xij, &r2);
            if (s->rg * s->rg - r2 > 0) {   /* 1st term */
                const double a = s->cofa[s->prop[i]] * (s->cofk) * (s->cofk);
                const double ratio = s->c.interaction_ratio[s->prop[i]][s->prop[j]];
                const double r = sqrt(r2);
                const double w = ratio * k_wg(s, r, s->rg);
                double fij[3];
                for (int d = 0; d < 3; ++d)
                    fij[d] = -a * (-s->gc[i][d]) * w / s->r2g * s->rg * (s->vol / s->dx);
                for (int p = 0; p < 3; ++p)
                    for (int q = 0; q < 3; ++q) st[p][q] += 1.0 * fij[p] * xij[q] / s->vol;
            }
            if (s->rg * s->rg - r2 > 0.0) {   /* 2nd term */
                const double a = s->cofa[s->prop[i]] * (s->cofk) * (s->cofk);
                const double ratio = s->c.interaction_ratio[s->prop[i]][s->prop[j]];
                const double r = sqrt(r2);
                const double dw = ratio * k_dwg(s, r, s->rg);
                const double gradw[3] = {dw * xij[0] / r, dw * xij[1] / r, dw * xij[2] / r};
                double gr = 0.0;
                for (int d = 0; d < 3; ++d) gr += (-s->gc[i][d]) * xij[d];
                double fij[3];
                for (int d = 0; d < 3; ++d) fij[d] = -a * (gr) * gradw[d] / s->r2g * s->rg * (s->vol / s->dx);
                for (int p = 0; p < 3; ++p)
                    for (int q = 0; q < 3; ++q) st[p][q] += 1.0 * fij[p] * xij[q] / s->vol;
            }
        }
        orc_virial_add(s, i, st);
    }
    for (int i = 0; i < s->n; ++i)   /* 3285-3294 */
        s->vpres[i] = s->dim == 2 ? -1.0 / 2.0 * (s->virial[i][0][0] + s->virial[i][1][1])
                                  : -1.0 / 3.0 * (s->virial[i][0][0] + s->virial[i][1][1] + s->virial[i][2][2]);
}

/* setInitialVelocityProfile, main.cpp:395-441 (constants 374-384).  Bar_Module: the beam's first
 * bending mode on the structure particles (its only call, main.cpp:571, is commented out, so it
 * is an explicit option here).  Turek_Hron: the parabolic inlet (x <= 0.01) and, while
 * Time < 0.7, the outlet band (x > 1.5) on the fluid particles -- called every step before
 * calculateWall (main.cpp:592-594).  Other modules: no body.                                  */
static double orc_beam_mode(double x)   /* compute_fx, main.cpp:387-392 */
{
    const double kL = 1.875, L = 0.20, k = kL / L;
    const double kx = k * x;
    const double term1 = (cos(kL) + cosh(kL)) * (cosh(kx) - cos(kx));
    const double term2 = (sin(kL) - sinh(kL)) * (sinh(kx) - sin(kx));
    return term1 + term2;
}

static void orc_velocity_profile(OrcState* s)
{
    if (s->c.module == MPH_MODULE_BAR) {
        const double K = 3.25e6, L = 0.20;
        for (int i = s->struct_b; i < s->struct_e; ++i) {
            const double rho = s->c.density[s->prop[i]];
            const double c0 = sqrt(K / rho);
            const double fx = orc_beam_mode(s->x0[i][0]);
            const double fL = orc_beam_mode(L);
            s->v[i][0] = 0.0;
            s->v[i][1] = 0.01 * c0 * fx / fL;
            s->v[i][2] = 0.0;
        }
    } else if (s->c.module == MPH_MODULE_TUREK_HRON) {
        const double YMIN = 0.0, YMAX = 0.41, UMAX = 1.0, H = YMAX - YMIN;
        for (int i = s->fluid_b; i < s->fluid_e; ++i) {
            const double x = s->x[i][0], y = s->x[i][1];
            if (x <= 0.01) {
                const double uy = y - YMIN;
                s->v[i][0] = (1.5 * 4.0 * UMAX / (H * H)) * uy * (H - uy);
                s->v[i][1] = 0.0;
                s->v[i][2] = 0.0;
            }
            if (x > 1.5 && s->time < 0.7) {
                const double uy = y - YMIN;
                s->v[i][0] = (4.0 * UMAX / (H * H)) * uy * (H - uy);
                s->v[i][1] = 0.0;
                s->v[i][2] = 0.0;
            }
        }
    }
}

static void orc_one_step(OrcState* s)   /* main.cpp:597-686 without I/O */
{
    if (s->c.module == MPH_MODULE_TUREK_HRON) orc_velocity_profile(s);   /* main.cpp:592-594 */
    orc_wall(s);
    orc_periodic(s);
    orc_reset_force(s);
    orc_reset_accel(s);
    orc_neighbor(s);
    orc_density_a(s);
    orc_gravity_center(s);
    orc_density_p(s);
    orc_divergence_p(s);
    orc_coefficients(s);
    orc_pressure_p(s);
    orc_pressure_a(s);
    orc_diffuse_interface(s);
    orc_viscosity(s);
    orc_gravity(s);
    orc_interface_force(s);
    orc_kick(s);
    orc_convection(s);
    const int sub = (int)(s->dt / s->edt + 0.5);
    for (int k = 0; k < sub; ++k) {
        orc_deformation(s);
        orc_stress(s);
        orc_stress_force(s);
        orc_update_elastic(s);
    }
    s->time += s->dt;
}

OrcState* orc_create(const MphConfig* cfg, int n, const int* property, const double* pos,
                     const double* pos0, const double* vel)
{
    OrcState* s = (OrcState*)calloc(1, sizeof(OrcState));
    s->c = *cfg;
    s->dim = cfg->dim;
    s->n = n;
    s->dx = cfg->particle_spacing;
    s->vol = s->dim == 2 ? s->dx * s->dx : s->dx * s->dx * s->dx;   /* main.cpp:805-809 */
    s->time = cfg->time;
    s->dt = cfg->dt;
    s->edt = cfg->elastic_dt;
    for (int d = 0; d < 3; ++d) { s->dmin[d] = cfg->domain_min[d]; s->dmax[d] = cfg->domain_max[d]; }
    memcpy(s->wall_c, cfg->wall_center, sizeof s->wall_c);
#define ALLOC(p, cnt) p = calloc((size_t)(cnt), sizeof(*(p)))
    ALLOC(s->prop, n); ALLOC(s->x, n); ALLOC(s->x0, n); ALLOC(s->v, n); ALLOC(s->f, n);
    ALLOC(s->acc, n); ALLOC(s->gc, n); ALLOC(s->mass, n); ALLOC(s->kappa, n); ALLOC(s->lambda, n);
    ALLOC(s->mu, n); ALLOC(s->young, n); ALLOC(s->dens_a, n); ALLOC(s->pres_a, n);
    ALLOC(s->vstrain, n); ALLOC(s->div_p, n); ALLOC(s->pres_p, n); ALLOC(s->lame_l, n);
    ALLOC(s->lame_m, n); ALLOC(s->normalizer, n); ALLOC(s->deform, n); ALLOC(s->strain, n);
    ALLOC(s->stress, n); ALLOC(s->ncount, n); ALLOC(s->sncount, n);
    ALLOC(s->virial, n); ALLOC(s->vpres, n);
    s->nlist = (int*)malloc(sizeof(int) * (size_t)n * MAXN);
    s->snlist = (int*)malloc(sizeof(int) * (size_t)n * MAXN);
    memcpy(s->prop, property, sizeof(int) * n);
    memcpy(s->x, pos, sizeof(v3) * n);
    memcpy(s->x0, pos0, sizeof(v3) * n);
    memcpy(s->v, vel, sizeof(v3) * n);
    /* class ranges, main.cpp:909-929 */
    s->fluid_b = s->fluid_e = s->struct_b = s->struct_e = s->wall_b = s->wall_e = -1;
    for (int i = 0; i < n; ++i) {
        const int t = s->prop[i];
        if (IS_FLUID(t)) { if (s->fluid_b == -1) s->fluid_b = i; s->fluid_e = i + 1; }
        else if (IS_STRUCT(t)) { if (s->struct_b == -1) s->struct_b = i; s->struct_e = i + 1; }
        else if (t >= 4 && t < 6) { if (s->wall_b == -1) s->wall_b = i; s->wall_e = i + 1; }
    }
    orc_init_weight(s);
    orc_init_fluid(s);
    orc_init_wall(s);
    orc_init_domain(s);
    ALLOC(s->cell_index, s->pow2); ALLOC(s->cell_particle, s->pow2);
    ALLOC(s->cell_begin, s->cell_total + 1); ALLOC(s->cell_end, s->cell_total + 1);
#undef ALLOC
    return s;
}

void orc_init(OrcState* s)   /* main.cpp:564-570 */
{
    orc_initial_neighbor(s);
    orc_neighbor(s);
    orc_density_a(s);
    orc_gravity_center(s);
    orc_density_p(s);
    orc_lame(s);
    orc_normalizer(s);
}

void orc_step(OrcState* s, int nsteps)
{
    for (int k = 0; k < nsteps; ++k) orc_one_step(s);
}

int orc_call(OrcState* s, const char* name)
{
    static const struct { const char* name; void (*fn)(OrcState*); } table[] = {
        {"calculateWall", orc_wall}, {"calculatePeriodicBoundary", orc_periodic},
        {"resetForce", orc_reset_force}, {"resetAccel", orc_reset_accel},
        {"calculateNeighbor", orc_neighbor}, {"calculateDensityA", orc_density_a},
        {"calculateGravityCenter", orc_gravity_center}, {"calculateDensityP", orc_density_p},
        {"calculateDivergenceP", orc_divergence_p}, {"calculatePhysicalCoefficients", orc_coefficients},
        {"calculatePressureP", orc_pressure_p}, {"calculatePressureA", orc_pressure_a},
        {"calculateDiffuseInterface", orc_diffuse_interface}, {"calculateViscosityV", orc_viscosity},
        {"calculateGravity", orc_gravity}, {"calculateInterfaceForce", orc_interface_force},
        {"calculateAcceleration", orc_kick}, {"calculateConvection", orc_convection},
        {"calculateElasticDeformationVector", orc_deformation}, {"calculateStress", orc_stress},
        {"calculateStressForce", orc_stress_force}, {"updateElasticPosition", orc_update_elastic},
        {"calculateVirialStressAtParticle", orc_virial},
        {"setInitialVelocityProfile", orc_velocity_profile},
    };
    for (size_t k = 0; k < sizeof table / sizeof table[0]; ++k)
        if (strcmp(name, table[k].name) == 0) { table[k].fn(s); return 0; }
    if (strcmp(name, "advanceTime") == 0) { s->time += s->dt; return 0; }
    return -1;
}

int orc_get(OrcState* s, const char* name, void* out)
{
    const int n = s->n;
    struct { const char* name; void* p; int w; int isint; } f[] = {
        {"Position", s->x, 3, 0}, {"InitialPosition", s->x0, 3, 0}, {"Velocity", s->v, 3, 0},
        {"Force", s->f, 3, 0}, {"Acceleration", s->acc, 3, 0}, {"GravityCenter", s->gc, 3, 0},
        {"DeformGradient", s->deform, 9, 0}, {"Strain", s->strain, 9, 0}, {"Stress", s->stress, 9, 0},
        {"Normalizer", s->normalizer, 9, 0}, {"PressureP", s->pres_p, 1, 0},
        {"PressureA", s->pres_a, 1, 0}, {"DensityA", s->dens_a, 1, 0}, {"VolStrainP", s->vstrain, 1, 0},
        {"DivergenceP", s->div_p, 1, 0}, {"Mass", s->mass, 1, 0}, {"Kappa", s->kappa, 1, 0},
        {"Lambda", s->lambda, 1, 0}, {"Mu", s->mu, 1, 0}, {"LambdaLames", s->lame_l, 1, 0},
        {"MuLames", s->lame_m, 1, 0}, {"NeighborCount", s->ncount, 1, 1},
        {"InitialStructureNeighborCount", s->sncount, 1, 1}, {"Property", s->prop, 1, 1},
        {"VirialStressAtParticle", s->virial, 9, 0}, {"VirialPressureAtParticle", s->vpres, 1, 0},
    };
    for (size_t k = 0; k < sizeof f / sizeof f[0]; ++k)
        if (strcmp(name, f[k].name) == 0) {
            memcpy(out, f[k].p, (size_t)n * f[k].w * (f[k].isint ? sizeof(int) : sizeof(double)));
            return n * f[k].w;
        }
    return -1;
}

int orc_neighbors(OrcState* s, int i, int* out)
{
    const int c = s->ncount[i];
    memcpy(out, s->nlist + (size_t)i * MAXN, sizeof(int) * (c < MAXN ? c : MAXN));
    return c;
}

int orc_scalars(OrcState* s, double* o)
{
    o[0] = s->n0a; o[1] = s->n0p; o[2] = s->swa; o[3] = s->swg; o[4] = s->swp; o[5] = s->swv;
    o[6] = s->r2g; o[7] = s->max_radius; o[8] = s->ra; o[9] = s->rg; o[10] = s->rp; o[11] = s->rv;
    o[12] = s->cofk; o[13] = s->vol; o[14] = s->dx; o[15] = s->dt; o[16] = s->edt;
    for (int d = 0; d < 3; ++d) { o[17 + d] = s->dmin[d]; o[20 + d] = s->dmax[d]; o[23 + d] = s->dw[d]; }
    for (int t = 0; t < NT; ++t) o[26 + t] = s->cofa[t];
    o[32] = s->cell_w;
    o[33] = s->cell_n[0]; o[34] = s->cell_n[1]; o[35] = s->cell_n[2];
    return 36;
}

double orc_time(OrcState* s) { return s->time; }
int orc_count(OrcState* s) { return s->n; }

void orc_set_threads(int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

void orc_destroy(OrcState* s)
{
    if (!s) return;
    void* ptrs[] = {s->prop, s->x, s->x0, s->v, s->f, s->acc, s->gc, s->mass, s->kappa, s->lambda,
                    s->mu, s->young, s->dens_a, s->pres_a, s->vstrain, s->div_p, s->pres_p,
                    s->lame_l, s->lame_m, s->normalizer, s->deform, s->strain, s->stress,
                    s->ncount, s->nlist, s->sncount, s->snlist, s->cell_index, s->cell_particle,
                    s->cell_begin, s->cell_end, s->virial, s->vpres};
    for (size_t k = 0; k < sizeof ptrs / sizeof ptrs[0]; ++k) free(ptrs[k]);
    free(s);
}
