// mph_host.cpp -- host layer of libmph_gpu.so: the reference's file formats and every constant
// it derives before the time loop.  Compiled with -ffp-contract=off: the derived constants are
// bit-identical to the reference's globals (checked by tests/test_host_io.py against
// oracle/_ref ref_scalars).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "mph_internal.h"

using namespace mph;

extern "C" int mph_config_sizeof(void) { return (int)sizeof(MphConfig); }

extern "C" int mph_abi_version(void) { return MPH_ABI_VERSION; }

extern "C" int mph_config_default(MphConfig* cfg, int dim, int module)
{
    if (!cfg || (dim != 2 && dim != 3) || module < 0 || module > MPH_MODULE_NONE) return MPH_ERR_ARG;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->dim = dim;
    cfg->module = module;
    cfg->dt = 1.0e100;          // main.cpp:91-92 static initialisers
    cfg->elastic_dt = 1.0e100;
    return MPH_OK;
}

// readDataFile, main.cpp:729-786: same keyword grammar (the sscanf format strings are the file
// format), first matching keyword wins, lines that match nothing are ignored.
extern "C" int mph_read_data_file(const char* path, MphConfig* c)
{
    if (!path || !c) return MPH_ERR_ARG;
    FILE* fp = std::fopen(path, "r");
    if (!fp) return MPH_ERR_IO;
    char buf[1024];
    double* d = c->density;
    double* k = c->bulk_modulus;
    double* bv = c->bulk_viscosity;
    double* sv = c->shear_viscosity;
    double* st = c->surface_tension;
    double* ym = c->young_modulus;
    double* pr = c->poisson_ratio;
    while (!std::feof(fp) && !std::ferror(fp)) {
        if (std::fgets(buf, sizeof(buf), fp) == nullptr) break;
        if (buf[0] == '#') continue;
        if (std::sscanf(buf, " Dt %lf", &c->dt) == 1) continue;
        if (std::sscanf(buf, " ElasticDt %lf", &c->elastic_dt) == 1) continue;
        if (std::sscanf(buf, " OutputInterval %lf", &c->output_interval) == 1) continue;
        if (std::sscanf(buf, " VtkOutputInterval %lf", &c->vtk_output_interval) == 1) continue;
        if (std::sscanf(buf, " EndTime %lf", &c->end_time) == 1) continue;
        if (std::sscanf(buf, " RadiusRatioA %lf", &c->radius_ratio_a) == 1) continue;
        if (std::sscanf(buf, " RadiusRatioP %lf", &c->radius_ratio_p) == 1) continue;
        if (std::sscanf(buf, " RadiusRatioV %lf", &c->radius_ratio_v) == 1) continue;
        if (std::sscanf(buf, " Density %lf %lf %lf %lf %lf %lf", d, d + 1, d + 2, d + 3, d + 4, d + 5) == 6) continue;
        if (std::sscanf(buf, " BulkModulus %lf %lf %lf %lf %lf %lf", k, k + 1, k + 2, k + 3, k + 4, k + 5) == 6) continue;
        if (std::sscanf(buf, " BulkViscosity %lf %lf %lf %lf %lf %lf", bv, bv + 1, bv + 2, bv + 3, bv + 4, bv + 5) == 6) continue;
        if (std::sscanf(buf, " ShearViscosity %lf %lf %lf %lf %lf %lf", sv, sv + 1, sv + 2, sv + 3, sv + 4, sv + 5) == 6) continue;
        if (std::sscanf(buf, " SurfaceTension %lf %lf %lf %lf", st, st + 1, st + 4, st + 5) == 4) continue;
        if (std::sscanf(buf, " YoungModulus %lf %lf %lf %lf", ym + 2, ym + 3, ym + 4, ym + 5) == 4) continue;
        if (std::sscanf(buf, " PoissonRatio %lf %lf %lf %lf ", pr + 2, pr + 3, pr + 4, pr + 5) == 4) continue;
        bool matched = false;
        for (int t = 0; t < kTypes && !matched; ++t) {
            char fmt[96];
            std::snprintf(fmt, sizeof(fmt), " InteractionRatio(Type%d) %%lf %%lf %%lf %%lf %%lf %%lf", t);
            double* r = c->interaction_ratio[t];
            matched = std::sscanf(buf, fmt, r, r + 1, r + 2, r + 3, r + 4, r + 5) == 6;
        }
        if (matched) continue;
        if (std::sscanf(buf, " Gravity %lf %lf %lf", c->gravity, c->gravity + 1, c->gravity + 2) == 3) continue;
        for (int w = 0; w < 2 && !matched; ++w) {
            const int t = 4 + w;
            const char* fmt = w == 0
                ? " Wall6  Center %lf %lf %lf Velocity %lf %lf %lf Omega %lf %lf %lf"
                : " Wall7  Center %lf %lf %lf Velocity %lf %lf %lf Omega %lf %lf %lf";
            double* C = c->wall_center[t];
            double* V = c->wall_velocity[t];
            double* O = c->wall_omega[t];
            matched = std::sscanf(buf, fmt, C, C + 1, C + 2, V, V + 1, V + 2, O, O + 1, O + 2) == 9;
        }
        // anything else: "Invalid line in data file" (main.cpp:768-770) -- ignored
    }
    std::fclose(fp);
    return MPH_OK;
}

// ---- binary grid (mph_write_grid_binary) -------------------------------------------------------
namespace {
constexpr char kGridMagic[8] = {'M', 'P', 'H', 'G', 'R', 'I', 'D', 'B'};
struct GridBinHeader {
    char magic[8];
    int32_t version, n;
    double time, dx, dmin[3], dmax[3];
};
static_assert(sizeof(GridBinHeader) == 80, "binary grid header layout");

bool is_grid_binary(const char* path, GridBinHeader* h)
{
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return false;
    GridBinHeader t;
    const bool ok = std::fread(&t, sizeof(t), 1, fp) == 1 && std::memcmp(t.magic, kGridMagic, 8) == 0 &&
                    t.version == 1 && t.n >= 0;
    std::fclose(fp);
    if (ok && h) *h = t;
    return ok;
}
}  // namespace

extern "C" int mph_write_grid_binary(const char* path, const MphConfig* c, int n, const int* prop,
                                     const double* pos, const double* pos0, const double* vel)
{
    if (!path || !c || n < 0 || (n > 0 && (!prop || !pos || !pos0 || !vel))) return MPH_ERR_ARG;
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return MPH_ERR_IO;
    GridBinHeader h{};
    std::memcpy(h.magic, kGridMagic, 8);
    h.version = 1;
    h.n = n;
    h.time = c->time;
    h.dx = c->particle_spacing;
    for (int d = 0; d < 3; ++d) { h.dmin[d] = c->domain_min[d]; h.dmax[d] = c->domain_max[d]; }
    bool ok = std::fwrite(&h, sizeof(h), 1, fp) == 1;
    ok = ok && std::fwrite(prop, sizeof(int), (size_t)n, fp) == (size_t)n;
    const int32_t pad = 0;
    if (n & 1) ok = ok && std::fwrite(&pad, sizeof(pad), 1, fp) == 1;
    for (const double* a : {pos, pos0, vel}) ok = ok && std::fwrite(a, sizeof(double) * 3, (size_t)n, fp) == (size_t)n;
    ok = std::fclose(fp) == 0 && ok;
    return ok ? MPH_OK : MPH_ERR_IO;
}

// readGridFile header, main.cpp:796-804
extern "C" int mph_read_grid_header(const char* path, MphConfig* c, int* n)
{
    if (!path || !c || !n) return MPH_ERR_ARG;
    GridBinHeader bh;
    if (is_grid_binary(path, &bh)) {
        c->time = bh.time;
        c->particle_spacing = bh.dx;
        for (int d = 0; d < 3; ++d) { c->domain_min[d] = bh.dmin[d]; c->domain_max[d] = bh.dmax[d]; }
        *n = bh.n;
        return MPH_OK;
    }
    FILE* fp = std::fopen(path, "r");
    if (!fp) return MPH_ERR_IO;
    char buf[1024];
    int rc = MPH_ERR_IO;
    if (std::fgets(buf, sizeof(buf), fp) && std::sscanf(buf, "%lf", &c->time) == 1 &&
        std::fgets(buf, sizeof(buf), fp) &&
        std::sscanf(buf, "%d  %lf  %lf %lf %lf  %lf %lf %lf", n, &c->particle_spacing,
                    &c->domain_min[0], &c->domain_max[0], &c->domain_min[1], &c->domain_max[1],
                    &c->domain_min[2], &c->domain_max[2]) == 8)
        rc = MPH_OK;
    std::fclose(fp);
    return rc;
}

// readGridFile body, main.cpp:896-904
extern "C" int mph_read_grid_particles(const char* path, int n, int* prop, double* pos, double* pos0,
                                       double* vel)
{
    if (!path || n < 0 || !prop || !pos || !pos0 || !vel) return MPH_ERR_ARG;
    GridBinHeader bh;
    if (is_grid_binary(path, &bh)) {
        if (bh.n != n) return MPH_ERR_ARG;
        FILE* fb = std::fopen(path, "rb");
        if (!fb) return MPH_ERR_IO;
        bool ok = std::fseek(fb, (long)sizeof(GridBinHeader), SEEK_SET) == 0;
        ok = ok && std::fread(prop, sizeof(int), (size_t)n, fb) == (size_t)n;
        int32_t pad;
        if (n & 1) ok = ok && std::fread(&pad, sizeof(pad), 1, fb) == 1;
        for (double* a : {pos, pos0, vel}) ok = ok && std::fread(a, sizeof(double) * 3, (size_t)n, fb) == (size_t)n;
        std::fclose(fb);
        return ok ? MPH_OK : MPH_ERR_IO;
    }
    FILE* fp = std::fopen(path, "r");
    if (!fp) return MPH_ERR_IO;
    char buf[1024];
    if (!std::fgets(buf, sizeof(buf), fp) || !std::fgets(buf, sizeof(buf), fp)) {
        std::fclose(fp);
        return MPH_ERR_IO;
    }
    int i = 0;
    for (; i < n; ++i) {
        if (std::fgets(buf, sizeof(buf), fp) == nullptr) break;
        double* x = pos + 3 * i;
        double* x0 = pos0 + 3 * i;
        double* v = vel + 3 * i;
        std::sscanf(buf, "%d  %lf %lf %lf %lf %lf %lf  %lf %lf %lf", prop + i, x, x + 1, x + 2, x0,
                    x0 + 1, x0 + 2, v, v + 1, v + 2);
    }
    std::fclose(fp);
    return i == n ? MPH_OK : MPH_ERR_IO;
}

// writeProfFile, main.cpp:957-982
extern "C" int mph_write_prof_arrays(const char* path, const MphConfig* c, double time, int n,
                                     const int* prop, const double* pos, const double* pos0,
                                     const double* vel)
{
    FILE* fp = std::fopen(path, "w");
    if (!fp) return MPH_ERR_IO;
    std::fprintf(fp, "%e\n", time);
    std::fprintf(fp, "%d %e %e %e %e %e %e %e\n", n, c->particle_spacing, c->domain_min[0],
                 c->domain_max[0], c->domain_min[1], c->domain_max[1], c->domain_min[2],
                 c->domain_max[2]);
    for (int i = 0; i < n; ++i) {
        const double* x = pos + 3 * i;
        const double* x0 = pos0 + 3 * i;
        const double* v = vel + 3 * i;
        std::fprintf(fp, "%d %e %e %e %e %e %e  %e %e %e\n", prop[i], x[0], x[1], x[2], x0[0], x0[1],
                     x0[2], v[0], v[1], v[2]);
    }
    std::fflush(fp);
    std::fclose(fp);
    return MPH_OK;
}

namespace {

// Formats the per-particle lines of one output section, line(i, buf) -> length, with the host's
// cores in blocks of consecutive particles and writes the blocks in order, so the bytes are those
// of the reference's sequential fprintf loop.  The reference's ASCII writers run at ~490 B per
// particle: at D1M one .vtk is ~0.7 GB of printf output.
template <class F>
void write_lines(FILE* fp, int n, F line)
{
    constexpr int kChunk = 1 << 16;
    const int hw = (int)std::thread::hardware_concurrency();
    const int nt = std::max(1, std::min(n / kChunk, std::min(hw > 0 ? hw : 1, 32)));
    auto fmt = [&](int b, int e, std::string& out) {
        char buf[192];
        out.clear();
        out.reserve((size_t)(e - b) * 40);
        for (int i = b; i < e; ++i) out.append(buf, (size_t)line(i, buf));
    };
    if (nt <= 1) {
        std::string s;
        fmt(0, n, s);
        std::fwrite(s.data(), 1, s.size(), fp);
        return;
    }
    std::vector<std::string> out(nt);
    for (int base = 0; base < n; base += nt * kChunk) {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) {
            const int b = base + t * kChunk, e = std::min(n, b + kChunk);
            if (b >= e) { out[t].clear(); continue; }
            th.emplace_back([&, t, b, e] { fmt(b, e, out[t]); });
        }
        for (auto& x : th) x.join();
        for (int t = 0; t < nt; ++t) std::fwrite(out[t].data(), 1, out[t].size(), fp);
    }
}

}  // namespace

// writeVtkFile, main.cpp:984-1189 (legacy ASCII; values printed as (float) with %e).  Same bytes
// as the reference (tests/test_gpu_parity.py checks the sha256 at step 0); the sections are
// formatted in parallel (write_lines).
extern "C" int mph_write_vtk_arrays(const char* path, int n, const int* prop, const double* pos,
                                    const double* pos0, const double* vel, const double* acc,
                                    const double* force, const double* stress, const double* strain,
                                    const int* isnc, const int* nc)
{
    FILE* fp = std::fopen(path, "w");
    if (!fp) return MPH_ERR_IO;
    std::vector<char> iobuf(1 << 22);
    std::setvbuf(fp, iobuf.data(), _IOFBF, iobuf.size());
    auto vec3 = [&](const double* a) {
        write_lines(fp, n, [a](int i, char* buf) {
            return std::snprintf(buf, 192, "%e %e %e\n", (float)a[3 * i], (float)a[3 * i + 1], (float)a[3 * i + 2]);
        });
    };
    auto ints = [&](const int* a) {
        write_lines(fp, n, [a](int i, char* buf) { return std::snprintf(buf, 192, "%d\n", a[i]); });
    };
    std::fprintf(fp, "# vtk DataFile Version 2.0\n");
    std::fprintf(fp, "Unstructured Grid Example\n");
    std::fprintf(fp, "ASCII\n");
    std::fprintf(fp, "DATASET UNSTRUCTURED_GRID\n");
    std::fprintf(fp, "POINTS %d float\n", n);
    vec3(pos);
    std::fprintf(fp, "CELLS %d %d\n", n, 2 * n);
    write_lines(fp, n, [](int i, char* buf) { return std::snprintf(buf, 192, "1 %d ", i); });
    std::fprintf(fp, "\n");
    std::fprintf(fp, "CELL_TYPES %d\n", n);
    write_lines(fp, n, [](int, char* buf) { buf[0] = '1'; buf[1] = ' '; return 2; });
    std::fprintf(fp, "\n");
    std::fprintf(fp, "\n");
    std::fprintf(fp, "POINT_DATA %d\n", n);
    std::fprintf(fp, "SCALARS label float 1\n");
    std::fprintf(fp, "LOOKUP_TABLE default\n");
    ints(prop);
    std::fprintf(fp, "\n");
    std::fprintf(fp, "\n");
    std::fprintf(fp, "VECTORS displacement float\n");
    write_lines(fp, n, [pos, pos0](int i, char* buf) {
        const double* x = pos + 3 * i;
        const double* x0 = pos0 + 3 * i;
        const double d[3] = {x[0] - x0[0], x[1] - x0[1], x[2] - x0[2]};
        return std::snprintf(buf, 192, "%e %e %e\n", (float)d[0], (float)d[1], (float)d[2]);
    });
    for (int pass = 0; pass < 2; ++pass) {
        const double* m = pass == 0 ? stress : strain;
        const char* tag = pass == 0 ? "stress" : "strain";
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                std::fprintf(fp, "\n");
                std::fprintf(fp, " SCALARS %s%d%d float \n", tag, a, b);
                std::fprintf(fp, "LOOKUP_TABLE default\n");
                const int k = 3 * a + b;
                write_lines(fp, n, [m, k](int i, char* buf) { return std::snprintf(buf, 192, "%e\n", (float)m[9 * i + k]); });
            }
    }
    std::fprintf(fp, "VECTORS velocity float\n");
    vec3(vel);
    std::fprintf(fp, "\n");
    std::fprintf(fp, "VECTORS accel float\n");
    vec3(acc);
    std::fprintf(fp, "\n");
    std::fprintf(fp, "SCALARS Initialneighbor float 1\n");
    std::fprintf(fp, "LOOKUP_TABLE default\n");
    ints(isnc);
    std::fprintf(fp, "SCALARS neighbor float 1\n");
    std::fprintf(fp, "LOOKUP_TABLE default\n");
    ints(nc);
    std::fprintf(fp, "VECTORS velocity float\n");
    vec3(vel);
    std::fprintf(fp, "\n");
    std::fprintf(fp, "VECTORS force float\n");
    vec3(force);
    std::fprintf(fp, "\n");
    std::fflush(fp);
    const bool ok = !std::ferror(fp);
    std::fclose(fp);
    return ok ? MPH_OK : MPH_ERR_IO;
}

// Binary alternative to writeVtkFile: the same point fields in a VTK XML
// UnstructuredGrid with raw appended data (UInt64 block headers, little endian), Float32 like the
// reference's (float)-rounded ASCII, stress/strain as 9-component tensors.  ~150 B per particle
// against ~490 B of ASCII, and no printf.
extern "C" int mph_write_vtu_arrays(const char* path, int n, const int* prop, const double* pos,
                                    const double* pos0, const double* vel, const double* acc,
                                    const double* force, const double* stress, const double* strain,
                                    const int* isnc, const int* nc)
{
    if (!path || n < 0) return MPH_ERR_ARG;
    struct Arr {
        const char* name;   // nullptr: the Points array
        const char* type;
        int ncomp;
        size_t bytes;
        std::function<void(char*)> fill;
    };
    const size_t N = (size_t)n;
    auto f32 = [N](const double* a, int w) {
        return [a, w, N](char* out) {
            float* o = (float*)out;
            for (size_t k = 0; k < N * w; ++k) o[k] = (float)a[k];
        };
    };
    auto i32 = [N](const int* a) { return [a, N](char* out) { std::memcpy(out, a, sizeof(int) * N); }; };
    std::vector<Arr> pd = {
        {"label", "Int32", 1, 4 * N, i32(prop)},
        {"displacement", "Float32", 3, 12 * N,
         [&](char* out) {
             float* o = (float*)out;
             for (size_t k = 0; k < 3 * N; ++k) o[k] = (float)(pos[k] - pos0[k]);
         }},
        {"stress", "Float32", 9, 36 * N, f32(stress, 9)},
        {"strain", "Float32", 9, 36 * N, f32(strain, 9)},
        {"velocity", "Float32", 3, 12 * N, f32(vel, 3)},
        {"accel", "Float32", 3, 12 * N, f32(acc, 3)},
        {"Initialneighbor", "Int32", 1, 4 * N, i32(isnc)},
        {"neighbor", "Int32", 1, 4 * N, i32(nc)},
        {"force", "Float32", 3, 12 * N, f32(force, 3)},
    };
    std::vector<Arr> geo = {
        {nullptr, "Float32", 3, 12 * N, f32(pos, 3)},
        {"connectivity", "Int32", 1, 4 * N,
         [N](char* out) {
             int* o = (int*)out;
             for (size_t k = 0; k < N; ++k) o[k] = (int)k;
         }},
        {"offsets", "Int32", 1, 4 * N,
         [N](char* out) {
             int* o = (int*)out;
             for (size_t k = 0; k < N; ++k) o[k] = (int)k + 1;
         }},
        {"types", "UInt8", 1, N, [N](char* out) { std::memset(out, 1, N); }},   // VTK_VERTEX
    };
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return MPH_ERR_IO;
    uint64_t off = 0;
    auto decl = [&](const Arr& a) {
        std::fprintf(fp, "        <DataArray type=\"%s\"", a.type);
        if (a.name) std::fprintf(fp, " Name=\"%s\"", a.name);
        if (a.ncomp > 1) std::fprintf(fp, " NumberOfComponents=\"%d\"", a.ncomp);
        std::fprintf(fp, " format=\"appended\" offset=\"%llu\"/>\n", (unsigned long long)off);
        off += sizeof(uint64_t) + a.bytes;
    };
    std::fprintf(fp, "<?xml version=\"1.0\"?>\n<VTKFile type=\"UnstructuredGrid\" version=\"1.0\" "
                     "byte_order=\"LittleEndian\" header_type=\"UInt64\">\n  <UnstructuredGrid>\n"
                     "    <Piece NumberOfPoints=\"%d\" NumberOfCells=\"%d\">\n      <PointData>\n", n, n);
    for (const Arr& a : pd) decl(a);
    std::fprintf(fp, "      </PointData>\n      <Points>\n");
    decl(geo[0]);
    std::fprintf(fp, "      </Points>\n      <Cells>\n");
    for (size_t k = 1; k < geo.size(); ++k) decl(geo[k]);
    std::fprintf(fp, "      </Cells>\n    </Piece>\n  </UnstructuredGrid>\n  <AppendedData encoding=\"raw\">\n   _");
    std::vector<char> buf;
    for (const std::vector<Arr>* list : {&pd, &geo})
        for (const Arr& a : *list) {
            const uint64_t nb = a.bytes;
            buf.resize(std::max<size_t>(a.bytes, 1));
            a.fill(buf.data());
            std::fwrite(&nb, sizeof(nb), 1, fp);
            std::fwrite(buf.data(), 1, a.bytes, fp);
        }
    std::fprintf(fp, "\n  </AppendedData>\n</VTKFile>\n");
    std::fflush(fp);
    const bool ok = !std::ferror(fp);
    std::fclose(fp);
    return ok ? MPH_OK : MPH_ERR_IO;
}

extern "C" int mph_derive_scalars(const MphConfig* cfg, double* out36)
{
    if (!cfg || !out36 || (cfg->dim != 2 && cfg->dim != 3) || !(cfg->particle_spacing > 0.0)) return MPH_ERR_ARG;
    mph::HostDerived h;
    mph::derive_constants(*cfg, h);
    mph::fill_scalars(h, *cfg, out36);
    return MPH_OK;
}

extern "C" int mph_structure_init(const MphConfig* cfg, int n, const int* prop, const double* pos0,
                                  int* isnc, double* normalizer, double* lame_l, double* lame_m)
{
    if (!cfg || n < 0 || (n > 0 && (!prop || !pos0))) return MPH_ERR_ARG;
    mph::HostDerived h;
    mph::derive_constants(*cfg, h);
    mph::StructureInit S;
    std::string err;
    const int rc = mph::build_structure(*cfg, h, n, prop, pos0, S, err);
    if (rc != MPH_OK) return rc;
    if (isnc) std::memset(isnc, 0, sizeof(int) * (size_t)n);
    if (normalizer) std::memset(normalizer, 0, sizeof(double) * 9 * (size_t)n);
    if (lame_l) std::memset(lame_l, 0, sizeof(double) * (size_t)n);
    if (lame_m) std::memset(lame_m, 0, sizeof(double) * (size_t)n);
    for (size_t s = 0; s < S.orig.size(); ++s) {
        const int i = S.orig[s];
        if (isnc) isnc[i] = S.count[s];
        if (normalizer) std::memcpy(normalizer + (size_t)9 * i, &S.normalizer[9 * s], sizeof(double) * 9);
        if (lame_l) lame_l[i] = S.lame_l[s];
        if (lame_m) lame_m[i] = S.lame_m[s];
    }
    return MPH_OK;
}

// setInitialVelocityProfile (main.cpp:395-441, case constants 374-392) on host arrays in the
// reference's layout.  Bar_Module: first bending mode of the L = 0.2 m beam on the structure
// particles, v_y = 0.01 c0 f(x0)/f(L), c0 = sqrt(K/rho).  Turek_Hron: the parabolic inlet profile
// on the fluid particles (x <= 0.01, and x > 1.5 while time < 0.7).  Other modules: no change.
namespace {
double beam_mode(double x)   // compute_fx, main.cpp:387-392
{
    const double kL = 1.875, L = 0.20, k = kL / L;
    const double kx = k * x;
    const double term1 = (std::cos(kL) + std::cosh(kL)) * (std::cosh(kx) - std::cos(kx));
    const double term2 = (std::sin(kL) - std::sinh(kL)) * (std::sinh(kx) - std::sin(kx));
    return term1 + term2;
}
}  // namespace

extern "C" int mph_velocity_profile_arrays(const MphConfig* c, double time, int n, const int* prop,
                                           const double* pos, const double* pos0, double* vel)
{
    if (!c || n < 0 || (n > 0 && (!prop || !pos || !pos0 || !vel))) return MPH_ERR_ARG;
    if (c->module == MPH_MODULE_BAR) {
        const double K = 3.25e6, L = 0.20;
        for (int i = 0; i < n; ++i) {
            if (!mph::is_struct(prop[i])) continue;
            const double rho = c->density[prop[i]];
            const double c0 = std::sqrt(K / rho);
            const double fx = beam_mode(pos0[3 * (size_t)i]);
            const double fL = beam_mode(L);
            vel[3 * (size_t)i] = 0.0;
            vel[3 * (size_t)i + 1] = 0.01 * c0 * fx / fL;
            vel[3 * (size_t)i + 2] = 0.0;
        }
    } else if (c->module == MPH_MODULE_TUREK_HRON) {
        const double ymin = 0.0, ymax = 0.41, umax = 1.0, h = ymax - ymin;
        for (int i = 0; i < n; ++i) {
            if (!mph::is_fluid(prop[i])) continue;
            const double x = pos[3 * (size_t)i], y = pos[3 * (size_t)i + 1];
            double* v = vel + 3 * (size_t)i;
            if (x <= 0.01) {
                const double uy = y - ymin;
                v[0] = (1.5 * 4.0 * umax / (h * h)) * uy * (h - uy);
                v[1] = 0.0;
                v[2] = 0.0;
            }
            if (x > 1.5 && time < 0.7) {
                const double uy = y - ymin;
                v[0] = (4.0 * umax / (h * h)) * uy * (h - uy);
                v[1] = 0.0;
                v[2] = 0.0;
            }
        }
    }
    return MPH_OK;
}

namespace mph {

// ---- derived constants: initializeWeight/Fluid/Wall/Domain (main.cpp:1191-1469) ------------

static double wa_ref(int dim, double swa, double r, double h)      // main.cpp:299-305
{
    const double hh = dim == 2 ? h * h : h * h * h;
    return 1.0 / swa * 1.0 / hh * (r / h) * (1.0 - (r / h)) * (1.0 - (r / h));
}
static double wp_ref(int dim, double swp, double r, double h)      // main.cpp:335-341
{
    const double hh = dim == 2 ? h * h : h * h * h;
    return 1.0 / swp * 1.0 / hh * ((1.0 - r / h) * (1.0 - r / h));
}

void derive_constants(const MphConfig& c, HostDerived& h)
{
    const int dim = c.dim;
    const double dx = c.particle_spacing;
    h.dx = dx;
    h.vol = dim == 2 ? dx * dx : dx * dx * dx;                 // main.cpp:805-809
    h.ra = c.radius_ratio_a * dx;                              // main.cpp:1193-1198
    h.rg = c.radius_ratio_a * dx;
    h.rp = c.radius_ratio_p * dx;
    h.rv = c.radius_ratio_v * dx;
    if (dim == 2) {                                            // main.cpp:1201-1206
        h.swa = 1.0 / 2.0 * 2.0 / 15.0 * M_PI / dx / dx;
        h.swg = 1.0 / 2.0 * 1.0 / 3.0 * M_PI / dx / dx;
        h.swp = 1.0 / 2.0 * 1.0 / 3.0 * M_PI / dx / dx;
        h.swv = 1.0 / 2.0 * 1.0 / 3.0 * M_PI / dx / dx;
        h.r2g = 1.0 / 2.0 * 1.0 / 30.0 * M_PI * h.rg * h.rg / dx / dx / h.swg;
    } else {                                                   // main.cpp:1208-1212
        h.swa = 1.0 / 3.0 * 1.0 / 5.0 * M_PI / dx / dx / dx;
        h.swg = 1.0 / 3.0 * 2.0 / 5.0 * M_PI / dx / dx / dx;
        h.swp = 1.0 / 3.0 * 2.0 / 5.0 * M_PI / dx / dx / dx;
        h.swv = 1.0 / 3.0 * 2.0 / 5.0 * M_PI / dx / dx / dx;
        h.r2g = 1.0 / 3.0 * 4.0 / 105.0 * M_PI * h.rg * h.rg / dx / dx / dx / h.swg;
    }
    for (int which = 0; which < 2; ++which) {                  // N0a 1216-1259, N0p 1261-1304
        const double R = which == 0 ? h.ra : h.rp;
        const int range = (int)(R / dx + 3.0);
        const int zr = dim == 2 ? 0 : range;
        double sum = 0.0;
        for (int ix = -range; ix <= range; ++ix)
            for (int iy = -range; iy <= range; ++iy)
                for (int iz = -zr; iz <= zr; ++iz) {
                    if (ix == 0 && iy == 0 && iz == 0) continue;
                    const double x = dx * ((double)ix), y = dx * ((double)iy), z = dx * ((double)iz);
                    const double r2 = dim == 2 ? x * x + y * y : x * x + y * y + z * z;
                    if (r2 <= R * R) {
                        const double r = std::sqrt(r2);
                        sum += which == 0 ? wa_ref(dim, h.swa, r, R) : wp_ref(dim, h.swp, r, R);
                    }
                }
        (which == 0 ? h.n0a : h.n0p) = sum;
    }
    double integN, integX;                                     // main.cpp:1329-1337
    if (dim == 2) { h.cofk = 0.350778153; integN = 0.024679383; integX = 0.226126699; }
    else { h.cofk = 0.326976006; integN = 0.021425779; integX = 0.233977488; }
    for (int t = 0; t < kTypes; ++t)                           // main.cpp:1339-1341
        h.cofa[t] = c.surface_tension[t] / ((h.rg / dx) * (integN + h.cofk * h.cofk * integX));
    std::memset(h.wall_rot, 0, sizeof(h.wall_rot));            // main.cpp:1374-1408
    for (int t = 4; t < 6; ++t) {
        const double* w = c.wall_omega[t];
        double nrm[3] = {0.0, 0.0, 0.0}, q[4];
        const double theta = std::fabs(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        if (theta != 0.0)
            for (int d = 0; d < 3; ++d) nrm[d] = w[d] / theta;
        for (int d = 0; d < 3; ++d) q[d] = nrm[d] * std::sin(theta * c.dt / 2.0);
        q[3] = std::cos(theta * c.dt / 2.0);
        double (*R)[3] = h.wall_rot[t];
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
    h.cell_w = dx;                                             // initializeDomain 1414-1440
    double cc[3];
    for (int d = 0; d < 3; ++d) { h.dmin[d] = c.domain_min[d]; h.dmax[d] = c.domain_max[d]; }
    cc[0] = std::round((h.dmax[0] - h.dmin[0]) / h.cell_w);
    cc[1] = std::round((h.dmax[1] - h.dmin[1]) / h.cell_w);
    cc[2] = dim == 2 ? 1 : std::round((h.dmax[2] - h.dmin[2]) / h.cell_w);
    for (int d = 0; d < 3; ++d) h.cell_n[d] = (int)cc[d];
    if (cc[0] != (double)h.cell_n[0] || cc[1] != (double)h.cell_n[1] || cc[2] != (double)h.cell_n[2])
        for (int d = 0; d < 3; ++d) h.dmax[d] = h.dmin[d] + h.cell_w * (double)h.cell_n[d];
    for (int d = 0; d < 3; ++d) h.dw[d] = h.dmax[d] - h.dmin[d];
    h.max_radius = 0.0;                                        // main.cpp:1460-1463
    const double radii[4] = {h.ra, h.rg, h.rp, h.rv};
    for (double r : radii) h.max_radius = r > h.max_radius ? r : h.max_radius;
}

void fill_scalars(const HostDerived& h, const MphConfig& c, double* o)
{
    o[0] = h.n0a; o[1] = h.n0p; o[2] = h.swa; o[3] = h.swg; o[4] = h.swp; o[5] = h.swv;
    o[6] = h.r2g; o[7] = h.max_radius; o[8] = h.ra; o[9] = h.rg; o[10] = h.rp; o[11] = h.rv;
    o[12] = h.cofk; o[13] = h.vol; o[14] = h.dx; o[15] = c.dt; o[16] = c.elastic_dt;
    for (int d = 0; d < 3; ++d) { o[17 + d] = h.dmin[d]; o[20 + d] = h.dmax[d]; o[23 + d] = h.dw[d]; }
    for (int t = 0; t < kTypes; ++t) o[26 + t] = h.cofa[t];
    o[32] = h.cell_w;
    o[33] = h.cell_n[0]; o[34] = h.cell_n[1]; o[35] = h.cell_n[2];
}

// Cell order of a z-slab context: (y, z, x) (perm 3) or (x, z, y) (perm 4), i.e. which of x and
// y is the contiguous axis.
// A wavefront is a run of consecutive sorted particles along the contiguous axis; the search
// takes its fast wave-uniform path only when every lane is a few cells clear of the periodic
// faces (DevParams.inner_lo/hi), so a contiguous axis whose particle runs reach a face (the
// bottom wall of a tank at the domain edge, say) slows every column that touches it.  Pick the
// axis with fewer particles within 2 rc of its faces, then the one with the longer runs.
int choose_cell_order(const HostDerived& h, int n, const double* pos, double rc)
{
    long near[2] = {0, 0};
    double lo[2] = {1e300, 1e300}, hi[2] = {-1e300, -1e300};
    for (int i = 0; i < n; ++i) {
        for (int d = 0; d < 2; ++d) {
            const double a = pos[3 * (size_t)i + d];
            if (a - h.dmin[d] < 2.0 * rc || h.dmax[d] - a < 2.0 * rc) ++near[d];
            lo[d] = std::min(lo[d], a);
            hi[d] = std::max(hi[d], a);
        }
    }
    if (near[0] != near[1]) return near[0] < near[1] ? 3 : 4;
    return (hi[0] - lo[0]) >= (hi[1] - lo[1]) ? 3 : 4;
}

// Origin of the GPU cell grid along axis d, in whole cells from dmin: the middle of the longest
// circular run of cells that hold none of the initial particles, when that run is at least
// 2 m + 2 cells (m = the stencil margin); else 0 (the grid starts at dmin).  A grid whose faces lie
// in empty space keeps the waves at a wall on a periodic face of the domain (the dam's bottom
// wall at y = 0) off the wrapped slow path of the search (DevParams.sinner_lo, seam_occ).
int choose_grid_origin(const HostDerived& h, int n, const double* pos, int d, int gc, int m)
{
    if (gc <= 0 || n <= 0) return 0;
    std::vector<char> occ((size_t)gc, 0);
    const double ginv = gc / h.dw[d];
    for (int i = 0; i < n; ++i) {
        double u = pos[3 * (size_t)i + d] - h.dmin[d];
        u -= h.dw[d] * std::floor(u / h.dw[d]);
        const int c = std::min(gc - 1, std::max(0, (int)std::floor(u * ginv)));
        occ[(size_t)c] = 1;
    }
    int first = -1;
    for (int c = 0; c < gc && first < 0; ++c)
        if (occ[(size_t)c]) first = c;
    if (first < 0) return 0;
    // only worth it when particles lie within the margin of a face of the domain (the waves there
    // take the wrapped search otherwise); a grid that already starts in empty space stays at dmin
    bool at_face = false;
    for (int c = 0; c < m && !at_face; ++c) at_face = occ[(size_t)c] || occ[(size_t)(gc - 1 - c)];
    if (!at_face) return 0;
    int best = 0, best_start = 0, run = 0, run_start = 0;
    for (int k = 1; k <= gc; ++k) {   // one lap from the first occupied cell
        const int c = (first + k) % gc;
        if (!occ[(size_t)c]) {
            if (run == 0) run_start = c;
            ++run;
        } else {
            if (run > best) { best = run; best_start = run_start; }
            run = 0;
        }
    }
    if (best < 2 * m + 2) return 0;
    return (best_start + best / 2) % gc;
}

// GPU linked-cell grid: cells of width >= rc/kReach along the two outer axes (a +-kReach stencil
// covers the acceptance sphere) and >= rc/sa along the contiguous axis (z in 3-D, y in 2-D;
// a +-sa stencil, scanned as one contiguous index range per column, so thinner cells there
// only sharpen the cutoff trimming of each column).  Cell counts divide the periodic width
// exactly; every axis needs enough cells that the stencil never visits a cell twice.
int choose_grid(const HostDerived& h, int dim, double rc, int sa, int gc[3], double ginv[3], std::string& err,
                int perm)
{
    const int ca = contig_axis(dim, perm);   // the contiguous (half-width) axis
    for (int d = 0; d < 3; ++d) {
        if (d == 2 && dim == 2) { gc[d] = 1; ginv[d] = 1.0 / h.dw[d]; continue; }
        // the domain rule is the one of rc/2 cells on every axis (>= 5 of them), whatever kReach
        if ((int)std::floor(h.dw[d] / (0.5 * rc * (1.0 + 1e-6))) < 5) {
            err = "domain axis " + std::to_string(d) + " narrower than 2.5 x cutoff";
            return MPH_ERR_DOMAIN;
        }
        const int reach = d == ca ? sa : kReach;
        const double target = rc / reach * (1.0 + 1e-6);
        const int nc = (int)std::floor(h.dw[d] / target);
        if (nc < 2 * reach + 1) {
            err = "domain axis " + std::to_string(d) + " narrower than 2.5 x cutoff";
            return MPH_ERR_DOMAIN;
        }
        gc[d] = nc;
        ginv[d] = (double)nc / h.dw[d];
    }
    return MPH_OK;
}

void make_dev_params(const MphConfig& c, const HostDerived& h, int n, int n_struct, DevParams& P)
{
    std::memset(&P, 0, sizeof(P));
    P.n = n;
    P.slab_axis = -1;
    P.dim = c.dim;
    P.module = c.module;
    P.wall_motion = c.wall_motion;
    {
        const double rp = h.rp, hdp = c.dim == 2 ? rp * rp : rp * rp * rp;
        P.cw_pair = (1.0 / h.swp) * (1.0 / hdp);   // as build_structure's per-pair weight
    }
    P.n_struct = n_struct;
    P.substeps = (int)(c.dt / c.elastic_dt + 0.5);
    for (int d = 0; d < 3; ++d) {
        P.dmin[d] = h.dmin[d];
        P.corg[d] = h.dmin[d];
        P.dw[d] = h.dw[d];
        P.hw[d] = 0.5 * h.dw[d];
        P.w075[d] = 0.75 * h.dw[d];
    }
    const double margin = 0.1 * h.dx;                          // MARGIN, main.cpp:116
    P.rc2 = (h.max_radius + margin) * (h.max_radius + margin);
    P.ra = h.ra; P.rg = h.rg; P.rp = h.rp; P.rv = h.rv;
    P.ra2 = h.ra * h.ra; P.rg2 = h.rg * h.rg; P.rp2 = h.rp * h.rp; P.rv2 = h.rv * h.rv;
    P.inv_ra = 1.0 / h.ra; P.inv_rg = 1.0 / h.rg; P.inv_rp = 1.0 / h.rp; P.inv_rv = 1.0 / h.rv;
    auto hd = [&](double r) { return c.dim == 2 ? r * r : r * r * r; };
    P.ca = 1.0 / h.swa * 1.0 / hd(h.ra);
    P.cda = P.ca / h.ra;
    P.cg = 1.0 / h.swg * 1.0 / hd(h.rg);
    P.cdg = P.cg * (-2.0 / h.rg);
    P.cp = 1.0 / h.swp * 1.0 / hd(h.rp);
    P.cdp = P.cp * (-2.0 / h.rp);
    P.cv = 1.0 / h.swv * 1.0 / hd(h.rv);
    P.cdv = P.cv * (-2.0 / h.rv);
    P.cw = (1.0 / h.swp) * (1.0 / hd(h.rp));
    P.n0a = h.n0a; P.n0p = h.n0p; P.r2g = h.r2g; P.cofk = h.cofk; P.dx = h.dx; P.vol = h.vol;
    P.dt = c.dt; P.edt = c.elastic_dt;
    P.cvis = c.dim == 2 ? 8.0 : 10.0;                          // main.cpp:2510-2512
    for (int d = 0; d < 3; ++d) P.gravity[d] = c.gravity[d];
    P.surface = 0;
    for (int t = 0; t < kTypes; ++t) {
        P.cofa[t] = h.cofa[t];
        if (h.cofa[t] != 0.0) P.surface = 1;
        P.density[t] = c.density[t];
        P.inv_density[t] = 1.0 / c.density[t];
        P.mass[t] = c.density[t] * h.vol;                      // main.cpp:2105
        P.inv_mass[t] = 1.0 / P.mass[t];
        P.bulk[t] = c.bulk_modulus[t];
        P.bulk_visc[t] = c.bulk_viscosity[t];
        for (int u = 0; u < kTypes; ++u) {
            P.ratio[t][u] = c.interaction_ratio[t][u];
            const double mi = c.shear_viscosity[t], mj = c.shear_viscosity[u];
            P.mu_ij[t][u] = 2.0 * (mi * mj) / (mi + mj);      // main.cpp:2505
        }
        for (int d = 0; d < 3; ++d) {
            P.wall_omega[t][d] = c.wall_omega[t][d];
            P.wall_vel[t][d] = c.wall_velocity[t][d];
            for (int e = 0; e < 3; ++e) P.wall_rot[t][d][e] = h.wall_rot[t][d][e];
        }
    }
}

// ---- elastic-solid initialisation (host, once): calculateInitialNeighbor (1497-1658),
//      calculateLamesconstant (2526-2540), calculateNormalizer (2544-2653) -------------------

static inline double mod_ref(double x, double w) { return x - w * std::floor(x / w); }
static inline double image_ref(double a, double b, double w)
{
    return mod_ref(a - b + 0.5 * w, w) - 0.5 * w;
}

// f(b, e) over [0, n) in contiguous chunks on the host's cores (the per-slot work of
// build_structure is independent, so results do not depend on the thread count).
template <class F>
static void parallel_ranges(int n, F f)
{
    const int hw = (int)std::thread::hardware_concurrency();
    const int nt = std::max(1, std::min({hw > 0 ? hw : 1, 32, n / 2048}));
    if (nt <= 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    const int chunk = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int b = t * chunk, e = std::min(n, b + chunk);
        if (b < e) th.emplace_back([&f, b, e] { f(b, e); });
    }
    for (auto& x : th) x.join();
}

int build_structure(const MphConfig& c, const HostDerived& h, int n, const int* prop,
                    const double* pos0, StructureInit& S, std::string& err, bool lists)
{
    S.orig.clear();
    for (int i = 0; i < n; ++i)
        if (is_struct(prop[i])) S.orig.push_back(i);
    const int ns = (int)S.orig.size();
    S.count.assign(ns, 0);
    S.offset.assign(ns + 1, 0);
    S.nbr.clear();
    S.normalizer.assign((size_t)ns * 9, 0.0);
    S.lame_l.assign(ns, 0.0);
    S.lame_m.assign(ns, 0.0);
    if (ns == 0) return MPH_OK;
    if (!lists) {
        S.offset.clear();
        S.in_offset.clear();
        S.in_nbr.clear();
        S.pair_out.clear();
        for (int s = 0; s < ns; ++s) {   // Lame constants, main.cpp:2533-2539
            const int t = prop[S.orig[s]];
            const double E = c.young_modulus[t], v = c.poisson_ratio[t];
            S.lame_l[s] = (E * v) / ((1.0 + v) * (1.0 - 2.0 * v));
            S.lame_m[s] = E / (2.0 * (1.0 + v));
        }
        return MPH_OK;
    }
    const int dim = c.dim;
    const double rc = h.max_radius + (0.1 * h.dx);
    const double rc2 = rc * rc;
    // bin structure particles on a coarse host grid (cell >= rc) over the periodic domain
    int gn[3];
    for (int d = 0; d < 3; ++d) {
        gn[d] = (d == 2 && dim == 2) ? 1 : std::max(1, (int)std::floor(h.dw[d] / rc));
        if (gn[d] > 1024) gn[d] = 1024;
    }
    auto cell_of = [&](const double* x, int d) {
        int k = (int)std::floor((x[d] - h.dmin[d]) / h.dw[d] * gn[d]);
        k %= gn[d];
        if (k < 0) k += gn[d];
        return k;
    };
    const size_t ncell = (size_t)gn[0] * gn[1] * gn[2];
    std::vector<int> head(ncell, -1), next(ns, -1);
    for (int s = ns - 1; s >= 0; --s) {
        const double* x = pos0 + 3 * S.orig[s];
        const size_t k = ((size_t)cell_of(x, 0) * gn[1] + cell_of(x, 1)) * gn[2] + cell_of(x, 2);
        next[s] = head[k];
        head[k] = s;
    }
    std::vector<std::vector<int>> rows(ns);
    std::vector<int> too_many(ns, 0);
    parallel_ranges(ns, [&](int sb, int se) {
    for (int s = sb; s < se; ++s) {
        const int i = S.orig[s];
        const double* xi = pos0 + 3 * i;
        const int c0 = cell_of(xi, 0), c1 = cell_of(xi, 1), c2 = cell_of(xi, 2);
        const int r0 = gn[0] >= 3 ? 1 : 0, r1 = gn[1] >= 3 ? 1 : 0, r2 = gn[2] >= 3 ? 1 : 0;
        std::vector<int>& row = rows[s];
        // visit each distinct neighbouring cell once (small grids: whole axis)
        auto axis_cells = [&](int ci, int r, int g, int* out) {
            int m = 0;
            if (g < 3) { for (int k = 0; k < g; ++k) out[m++] = k; return m; }
            for (int o = -r; o <= r; ++o) out[m++] = ((ci + o) % g + g) % g;
            return m;
        };
        int buf0[1024], buf1[1024], buf2[1024];
        const int m0 = axis_cells(c0, r0, gn[0], buf0);
        const int m1 = axis_cells(c1, r1, gn[1], buf1);
        const int m2 = axis_cells(c2, r2, gn[2], buf2);
        for (int a = 0; a < m0; ++a)
            for (int b = 0; b < m1; ++b)
                for (int e = 0; e < m2; ++e) {
                    const size_t k = ((size_t)buf0[a] * gn[1] + buf1[b]) * gn[2] + buf2[e];
                    for (int t = head[k]; t >= 0; t = next[t]) {
                        const int j = S.orig[t];
                        if (j == i) continue;
                        const double* xj = pos0 + 3 * j;
                        double q[3];
                        q[0] = image_ref(xj[0], xi[0], h.dw[0]);
                        q[1] = image_ref(xj[1], xi[1], h.dw[1]);
                        q[2] = dim == 2 ? 0.0 : image_ref(xj[2], xi[2], h.dw[2]);  // main.cpp:1605
                        const double q2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2];
                        if (q2 <= rc2) row.push_back(t);
                    }
                }
        std::sort(row.begin(), row.end());
        too_many[s] = (int)row.size() >= kMaxNeighbor;
    }
    });
    for (int s = 0; s < ns; ++s)
        if (too_many[s]) {
            err = "structure particle " + std::to_string(S.orig[s]) + " has >= 512 initial neighbours";
            return MPH_ERR_NEIGHBOR_OVERFLOW;
        }
    for (int s = 0; s < ns; ++s) {
        S.count[s] = (int)rows[s].size();
        S.offset[s + 1] = S.offset[s] + S.count[s];
    }
    S.nbr.resize(S.offset[ns]);
    for (int s = 0; s < ns; ++s)
        std::copy(rows[s].begin(), rows[s].end(), S.nbr.begin() + S.offset[s]);
    // transpose (incoming list) for the gather form of calculateStressForce's scatter
    S.in_offset.assign(ns + 1, 0);
    for (int s = 0; s < ns; ++s)
        for (int t : rows[s]) S.in_offset[t + 1]++;
    for (int s = 0; s < ns; ++s) S.in_offset[s + 1] += S.in_offset[s];
    S.in_nbr.assign(S.in_offset[ns], 0);
    std::vector<int> fill(S.in_offset.begin(), S.in_offset.end() - 1);
    for (int s = 0; s < ns; ++s)
        for (int t : rows[s]) S.in_nbr[fill[t]++] = s;
    // Lame constants, main.cpp:2533-2539
    for (int s = 0; s < ns; ++s) {
        const int t = prop[S.orig[s]];
        const double E = c.young_modulus[t], v = c.poisson_ratio[t];
        S.lame_l[s] = (E * v) / ((1.0 + v) * (1.0 - 2.0 * v));
        S.lame_m[s] = E / (2.0 * (1.0 + v));
    }
    // Normalizer: 3x3 accumulation in both dims (TWO_DIMENSION typo, main.cpp:2545), then the
    // 2x2 inverse with identity fallback (2-D) or cofactor inverse without fallback (3-D)
    const double rp = h.rp;
    const double hd = dim == 2 ? rp * rp : rp * rp * rp;
    parallel_ranges(ns, [&](int sb, int se) {
    for (int s = sb; s < se; ++s) {
        const int i = S.orig[s];
        double N[3][3] = {{0.0}};
        for (int k = S.offset[s]; k < S.offset[s + 1]; ++k) {
            const int j = S.orig[S.nbr[k]];
            double x0[3];
            for (int d = 0; d < 3; ++d) x0[d] = image_ref(pos0[3 * j + d], pos0[3 * i + d], h.dw[d]);
            double r2 = 0.0;
            for (int d = 0; d < (dim == 2 ? 2 : 3); ++d) r2 += x0[d] * x0[d];
            const double q = std::sqrt(r2) / rp;
            const double w = (1.0 / h.swp) * (1.0 / hd) * ((1.0 - q) * (1.0 - q));
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) N[a][b] += w * x0[a] * x0[b];
        }
        if (dim == 2) {
            const double a = N[0][0], b = N[0][1], cc = N[1][0], d = N[1][1];
            const double det = a * d - b * cc;
            if (det != 0.0) {
                N[0][0] = d / det; N[0][1] = -b / det; N[1][0] = -cc / det; N[1][1] = a / det;
            } else {
                N[0][0] = 1.0; N[0][1] = 0.0; N[1][0] = 0.0; N[1][1] = 1.0;
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
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) N[a][b] = adj[a][b] / det;
            }
        }
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) S.normalizer[(size_t)s * 9 + 3 * a + b] = N[a][b];
    }
    });
    // per-pair constants of the fixed Lagrangian neighbourhood: x0_ij and weight(x0_ij)
    auto pair = [&](int s, int t, double* out4) {
        const int i = S.orig[s], j = S.orig[t];
        double x0[3] = {0.0, 0.0, 0.0};
        for (int d = 0; d < dim; ++d) x0[d] = image_ref(pos0[3 * j + d], pos0[3 * i + d], h.dw[d]);
        double r2 = 0.0;
        for (int d = 0; d < dim; ++d) r2 += x0[d] * x0[d];
        const double q = std::sqrt(r2) / rp;
        out4[0] = x0[0]; out4[1] = x0[1]; out4[2] = x0[2];
        out4[3] = (1.0 / h.swp) * (1.0 / hd) * ((1.0 - q) * (1.0 - q));
    };
    S.pair_out.resize((size_t)S.nbr.size() * 4);
    parallel_ranges(ns, [&](int sb, int se) {
        for (int s = sb; s < se; ++s)
            for (int k = S.offset[s]; k < S.offset[s + 1]; ++k) pair(s, S.nbr[k], &S.pair_out[(size_t)k * 4]);
    });
    return MPH_OK;
}

}  // namespace mph
