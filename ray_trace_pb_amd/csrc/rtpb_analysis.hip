// rtpb_analysis.hip -- device analysis around the trace: intersect_rays
// (RT:164-238), per-group spot statistics, the fused spot-diagram sweep (generate + trace + reduce),
// and griddata-style interpolation of pupil phases onto a grid.
#include "rtpb_internal.h"

#include <algorithm>
#include <array>
#include <map>

using namespace rtpbi;

namespace {

// intersect_rays (RT:164-238): closest-approach solve from the first non-singular 2x2 sub-system,
// verified to 1e-12.  NaN determinants count as "non-zero" exactly like numpy's truthiness.
struct IsectArgs {
    const void* __restrict__ r1;
    const void* __restrict__ r2;
    void* __restrict__ out;
    int64_t n, n1, n2;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void intersect_kernel(IsectArgs a) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= a.n) return;
    const T* p = static_cast<const T*>(a.r1) + (a.n1 == 1 ? 0 : i) * 8;
    const T* q = static_cast<const T*>(a.r2) + (a.n2 == 1 ? 0 : i) * 8;
    const double x1 = p[0], y1 = p[1], z1 = p[2], dx1 = p[3], dy1 = p[4], dz1 = p[5];
    const double x2 = q[0], y2 = q[1], z2 = q[2], dx2 = q[3], dy2 = q[4], dz2 = q[5];
    const double nan = qnan<double>();
    const double det_xz = dx2 * dz1 - dz2 * dx1, det_xy = dx2 * dy1 - dy2 * dx1, det_yz = dz2 * dy1 - dy2 * dz1;
    double s = nan;
    if (det_xz != 0.0) s = ((z2 - z1) * dx1 - (x2 - x1) * dz1) / det_xz;
    else if (det_xy != 0.0) s = ((y2 - y1) * dx1 - (x2 - x1) * dy1) / det_xy;
    else if (det_yz != 0.0) s = ((y2 - y1) * dz1 - (z2 - z1) * dy1) / det_yz;
    double t;
    if (dz1 != 0.0) t = (z2 + s * dz2 - z1) / dz1;
    else if (dy1 != 0.0) t = (y2 + s * dy2 - y1) / dy1;
    else t = (x2 + s * dx2 - x1) / dx1;
    double o[3] = {x1 + t * dx1, y1 + t * dy1, z1 + t * dz1};
    const double e[3] = {o[0] - (x2 + s * dx2), o[1] - (y2 + s * dy2), o[2] - (z2 + s * dz2)};
    // numpy.max over the 3 |differences| propagates NaN, and NaN > 1e-12 is false
    double m = tabs(e[0]);
    for (int k = 1; k < 3; ++k) {
        const double v = tabs(e[k]);
        if (is_nan(m)) break;
        if (is_nan(v) || v > m) m = v;
    }
    if (m > 1e-12) o[0] = o[1] = o[2] = nan;
    T* out = static_cast<T*>(a.out) + i * 3;
    out[0] = T(o[0]); out[1] = T(o[1]); out[2] = T(o[2]);
}

// Spot statistics of one history plane, per contiguous group of `gsize` rays (per
// (field, wavelength) spot diagrams).  Rays whose x or y is not finite are skipped.  Deterministic:
// pass 1 reduces each 256-ray tile of a group in a fixed tree order into partials[group][tile];
// pass 2 sums a group's partials in a fixed order.  Stats: n, Sx, Sy, Sz, Sxx, Syy, Sxy.
constexpr int kStats = 7;
struct SpotArgs {
    const void* __restrict__ plane;
    double* __restrict__ partials;
    double* __restrict__ stats;
    int64_t gsize, ngroups, tiles;
};

// Sums of R values over a block's 256 lanes in one fixed tree order -- red[t] += red[t + w] for t < w, w = 128, 64,
// ..., 1 -- valid in thread 0.  The two levels that cross waves go through LDS (buf rows, slots 64..255; two
// barriers), the six inside wave 0 through lane shuffles: the same additions of the same operands, without the
// barrier, store and load of every level of an all-LDS tree.
template <int R>
__device__ __forceinline__ void block_tree_sum(double (&v)[R], double (*buf)[kBlock]) {
    static_assert(kBlock == 256, "four waves");
    const int t = threadIdx.x;
    if (t >= 128) {
#pragma unroll
        for (int j = 0; j < R; ++j) buf[j][t] = v[j];
    }
    __syncthreads();
    if (t < 128) {
#pragma unroll
        for (int j = 0; j < R; ++j) v[j] = v[j] + buf[j][t + 128];
        if (t >= 64) {
#pragma unroll
            for (int j = 0; j < R; ++j) buf[j][t] = v[j];
        }
    }
    __syncthreads();
    if (t < 64) {
#pragma unroll
        for (int j = 0; j < R; ++j) v[j] = v[j] + buf[j][t + 64];
        // lanes >= w add values no later level reads
#pragma unroll
        for (int w = 32; w > 0; w >>= 1) {
#pragma unroll
            for (int j = 0; j < R; ++j) v[j] = v[j] + __shfl_down(v[j], w, 64);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void spot_partial_kernel(SpotArgs a) {
    __shared__ double red[kStats][kBlock];
    const int64_t g = blockIdx.y, tile = blockIdx.x;
    const int64_t j = tile * kBlock + threadIdx.x;
    double v[kStats] = {0, 0, 0, 0, 0, 0, 0};
    if (j < a.gsize) {
        const T* r = static_cast<const T*>(a.plane) + (g * a.gsize + j) * 8;
        const double x = r[0], y = r[1], z = r[2];
        if (x - x == 0.0 && y - y == 0.0) {
            v[0] = 1.0; v[1] = x; v[2] = y; v[3] = z; v[4] = x * x; v[5] = y * y; v[6] = x * y;
        }
    }
    block_tree_sum<kStats>(v, red);
    if (threadIdx.x == 0) {
        for (int k = 0; k < kStats; ++k) a.partials[(g * a.tiles + tile) * kStats + k] = v[k];
    }
}

__global__ __launch_bounds__(kBlock) void spot_final_kernel(SpotArgs a) {
    __shared__ double red[kStats][kBlock];
    const int64_t g = blockIdx.x;
    double v[kStats] = {0, 0, 0, 0, 0, 0, 0};
    for (int64_t t = threadIdx.x; t < a.tiles; t += kBlock)
        for (int k = 0; k < kStats; ++k) v[k] += a.partials[(g * a.tiles + t) * kStats + k];
    for (int k = 0; k < kStats; ++k) red[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int k = 0; k < kStats; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < kStats) a.stats[g * kStats + threadIdx.x] = red[threadIdx.x][0];
}

// Spot-diagram sweep, fused (C5).  Group g is the fan get_ray_fan(pt_g, ..., wl_g)
// (RT:45-96, same per-ray arithmetic as ray_fan_kernel, angles from the caller's tables); each ray is
// generated in registers, traced through the plan keeping only its final state, and reduced into the
// same 256-ray tile partials as spot_partial_kernel.  spot_final_kernel then produces statistics
// bit-identical to generating, tracing (planes='final') and reducing separately -- without the
// 3 x 64 B per ray of HBM traffic and the launches in between.
struct SweepArgs {
    const DevSurface<double>* __restrict__ surf;
    const DevMaterial<double>* __restrict__ mats;
    const double* __restrict__ table;
    const double2* __restrict__ tab;    // (cos, sin): thetas [n_thetas], then phis [nphis]
    const double* __restrict__ grp;     // per group: x, y, z, wavelength
    const double* __restrict__ gn;      // FEAT bit 4: per group, n of the S+1 materials at its wavelength, then
                                        // per surface n_s / n_s+1, 1 / n_s+1 and host_rcp_ok(n_s+1) (0 / 1)
    const int32_t* __restrict__ gidx;   // single rows: the group of block row y; bundle rows: see rows
    const int32_t* __restrict__ rows;   // bundle rows: (offset into gidx, number of groups) of block row y
    double* __restrict__ partials;
    int64_t n_thetas, nphis, gsize, tiles;
    double c[3], ex[3], ey[3];
    int32_t nsurf;
    // j / n_thetas as (j * nt_mul) >> nt_shift for j < 2^31 (nt_mul != 0, see sweep_divisor), else int64 division
    uint32_t nt_mul;
    int32_t nt_shift;
};

template <typename TS>
__device__ __forceinline__ double stored(double v) { return static_cast<double>(static_cast<TS>(v)); }

// kSweepRays rays per lane, traced side by side: each surface runs one surface_step instantiation per ray in one
// straight-line region (inside one run of equal surface codes), so independent dependency chains interleave (two:
// -6 % vs one ray per lane); each ray's 256-ray tile is reduced separately, with the same tree as
// spot_partial_kernel.  Single rows: block b covers tiles kSweepRays*b ... of one group.
// BUNDLE rows (round 5): up to kMaxBundle groups of one field point (a multiple of kSweepRays: 2, 4, 6 or 8) -- the same
// fan at several wavelengths.  Block b covers tile b of every group of the bundle: each lane generates its ray once
// and, when the first surface refracts (Flat / Sphere), runs the part of that surface that does not depend on the
// wavelength once (intersection, normal, front-side and on-surface tests, tangent basis: surface_step_pair's split)
// into LDS; then, kSweepRays groups at a time, it refracts the shared state with each group's Snell ratio
// (snell_apply) and traces those rays side by side through the other surfaces.  A field point's leftover groups run
// in single rows.
#ifndef RTPB_SWEEP_RPL
#define RTPB_SWEEP_RPL 2
#endif
constexpr int kSweepRays = RTPB_SWEEP_RPL;         // rays per lane (tiles per block)
// groups per bundle row: a multiple of kSweepRays (each pass of a row traces kSweepRays of its groups)
constexpr int kMaxBundle = 8 - 8 % kSweepRays;
constexpr int kStateRows = 11;                     // bundle state per lane: x y z, N, c, c . d, N . d

// Occupancy: held to >= 6 waves per SIMD (<= 80 VGPRs).  Round 3 measured 7 best (2.4 % faster than the natural
// 83 VGPRs / 5 waves, experiments/ab_sweep_wpe*.log); with round 4's lens instantiation, fixup-free quotients and
// x x + y y carry the sweep runs 0.379 s at 6, 0.384 s at 7, 0.401 s at 8 (profiles/r04/e/, one process,
// bit-identical); round 5's pair rows: 0.345 s at 6, 0.348 s at 5, 0.353 s at 7 (profiles/r05/g).  Bundle rows hold
// 26 KB of LDS per block (the state, and the reduction two statistics at a time), so 6 blocks fit a CU's 160 KB.
// RTPB_SWEEP_WPE overrides it (A/B builds).
#ifndef RTPB_SWEEP_WPE
#define RTPB_SWEEP_WPE 6
#endif
#define RTPB_SWEEP_ATTR __attribute__((amdgpu_waves_per_eu(RTPB_SWEEP_WPE, 8)))
template <typename TS, int FEAT, bool BUNDLE>
__global__ __launch_bounds__(kBlock) RTPB_SWEEP_ATTR void sweep_kernel(SweepArgs a) {
    static_assert(!BUNDLE || (FEAT & 16) != 0, "bundles: host-evaluated media");
    constexpr int kRedRows = BUNDLE ? 2 : kStats;
    __shared__ double red[kRedRows][kBlock];
    __shared__ double state[BUNDLE ? kStateRows : 1][kBlock];
    const int tid = threadIdx.x;
    auto gen = [&](int64_t j, const double* gp) {
        const int64_t jj = j < a.gsize ? j : 0;
        int64_t it, ip;
        if (a.nt_mul != 0) {
            const uint32_t x = static_cast<uint32_t>(jj);
            const uint32_t qt = static_cast<uint32_t>((uint64_t(x) * a.nt_mul) >> a.nt_shift);
            ip = qt;
            it = x - qt * static_cast<uint32_t>(a.n_thetas);
        } else {
            it = jj % a.n_thetas;
            ip = jj / a.n_thetas;
        }
        const double2 t = a.tab[it], ph = a.tab[a.n_thetas + ip];
        const double ct = t.x, st = t.y, cp = ph.x, sp = ph.y;
        Ray<double> r;
        r.x = stored<TS>(gp[0]); r.y = stored<TS>(gp[1]); r.z = stored<TS>(gp[2]);
        r.dx = stored<TS>(a.c[0] * ct + a.ex[0] * cp * st + a.ey[0] * sp * st);
        r.dy = stored<TS>(a.c[1] * ct + a.ex[1] * cp * st + a.ey[1] * sp * st);
        r.dz = stored<TS>(a.c[2] * ct + a.ex[2] * cp * st + a.ey[2] * sp * st);
        r.ph = 0.0;
        r.wl = stored<TS>(gp[3]);
        return r;
    };
    const cptr<DevSurface<double>> surf = (cptr<DevSurface<double>>)(a.surf);
    const cptr<DevMaterial<double>> mats = (cptr<DevMaterial<double>>)(a.mats);
    const cptr<double> table = (cptr<double>)(a.table);
    int64_t grp[kSweepRays], tile[kSweepRays];
    Ray<double> r[kSweepRays];
    // one wavelength per group: with FEAT bit 4 the host has evaluated every material at it (the kernel's own
    // material_n, see rtpb_spot_sweep) and the values arrive as scalar loads; without it (single rows only) every ray
    // of the block has the group's wavelength, so the per-wavelength values of ray 0 serve both
    Rcp<double> iwl[kSweepRays];
    cptr<double> gn[kSweepRays];
    double n_cur[kSweepRays];
    // the group's wavelength (not r[0].wl: a row kill fills the ray's wavelength with NaN too, and the single rows'
    // second ray takes ray 0's n)
    double wl0 = 0.0;
    auto mat_n = [&](int q, int k) -> double {
        if constexpr ((FEAT & 16) != 0) return gn[q][k];
        else return material_n<double, (FEAT & 2) != 0>(load_material<double>(mats + k), wl0, table);
    };
    // the surface's descriptor for ray q: with host-evaluated media, the Snell ratio and 1 / n2 of q's group (IEEE
    // division on the host)
    auto surface_for = [&](int q, int k, const DevSurface<double>& base) {
        DevSurface<double> sd = base;
        if constexpr ((FEAT & 16) != 0) {
            sd.nr = gn[q][a.nsurf + 1 + k];
            sd.rn2 = gn[q][2 * a.nsurf + 1 + k];
            sd.rcp_ok = (sd.rcp_ok & ~(4 | 8)) | 4 | (gn[q][3 * a.nsurf + 1 + k] != 0.0 ? 8 : 0);
        }
        return sd;
    };
    auto code_of = [&](int k) { return surface_code<double>((surf + k)->kind, (surf + k)->rcp_ok); };
    constexpr int kMode = kPosOnly | ((FEAT & 16) != 0 ? kUniMedia : 0);
    // the statistics read only the final positions: the steps run with kPosOnly semantics (no TIR fill of the
    // position -- the next surface's intersection makes it NaN, and the final plane gets the rule in reduce), and a
    // run of axial spheres carries x x + y y of each intersection point into the next sphere's quadratic.
    // Runs of consecutive surfaces of one (kind, axial) code: each run loops inside one instantiation of the surface
    // step, so the rays' registers carry from surface to surface without the copies a per-surface join of the kind
    // branches needs (the ODT path of C5: 12 axial spheres, a lens, a flat = 3 runs).
    double rxy[kSweepRays];
    auto trace_from = [&](int s) {
        while (s < a.nsurf) {
            const int code = code_of(s);
            dispatch_code<(FEAT & 1) != 0>(code, [&](auto kind, auto geo) {
                constexpr int K = decltype(kind)::value;
                constexpr int A = decltype(geo)::value;
                constexpr bool kCarry = K == SPHERE && A == kGeoAxial;
                if constexpr (kCarry) {
#pragma unroll
                    for (int q = 0; q < kSweepRays; ++q) rxy[q] = r[q].x * r[q].x + r[q].y * r[q].y;
                }
                do {
                    const DevSurface<double> base = load_surface<double>(surf + s);
                    double n_next[kSweepRays];
#pragma unroll
                    for (int q = 0; q < kSweepRays; ++q) n_next[q] = (BUNDLE || q == 0) ? mat_n(q, s + 1) : n_next[0];
                    auto none = [](const Ray<double>&) {};
                    Ray<double> o[kSweepRays];
#pragma unroll
                    for (int q = 0; q < kSweepRays; ++q) {
                        const DevSurface<double> sd = (BUNDLE || q == 0) ? surface_for(q, s, base)
                                                                         : surface_for(0, s, base);
                        surface_step<double, K, A, kMode>(sd, r[q], n_cur[q], n_next[q], iwl[q], none, o[q],
                                                          static_cast<GuardBranch*>(nullptr),
                                                          kCarry ? &rxy[q] : nullptr);
                    }
#pragma unroll
                    for (int q = 0; q < kSweepRays; ++q) {
                        r[q] = o[q];
                        n_cur[q] = n_next[q];
                    }
                    ++s;
                } while (s < a.nsurf && code_of(s) == code);
            });
        }
    };
    // one ray's contribution to its group's tile partial: spot_partial_kernel's tree (block_tree_sum), kRedRows
    // statistics at a time
    auto reduce = [&](const Ray<double>& rr, bool ok, int64_t g, int64_t t) {
        double v[kStats] = {0, 0, 0, 0, 0, 0, 0};
        // the reference's position rule of the last surface (RT:1221 / RT:1289; a PerfectLens's after-plane
        // propagation gives a NaN position for a NaN direction by itself): NaN direction -> no spot point
        if (ok && !is_nan(rr.dx)) {
            const double x = stored<TS>(rr.x), y = stored<TS>(rr.y), z = stored<TS>(rr.z);
            if (x - x == 0.0 && y - y == 0.0) {
                v[0] = 1.0; v[1] = x; v[2] = y; v[3] = z; v[4] = x * x; v[5] = y * y; v[6] = x * y;
            }
        }
#pragma unroll
        for (int k0 = 0; k0 < kStats; k0 += kRedRows) {
            double u[kRedRows];
#pragma unroll
            for (int j = 0; j < kRedRows; ++j) u[j] = k0 + j < kStats ? v[k0 + j] : 0.0;
            block_tree_sum<kRedRows>(u, red);
            if (tid == 0 && t < a.tiles) {
#pragma unroll
                for (int j = 0; j < kRedRows; ++j)
                    if (k0 + j < kStats) a.partials[(g * a.tiles + t) * kStats + k0 + j] = u[j];
            }
        }
    };
    if constexpr (!BUNDLE) {
#pragma unroll
        for (int q = 0; q < kSweepRays; ++q) {
            grp[q] = a.gidx[blockIdx.y];
            tile[q] = kSweepRays * int64_t(blockIdx.x) + q;
            r[q] = gen(tile[q] * kBlock + tid, a.grp + 4 * grp[q]);
        }
        wl0 = r[0].wl;
#pragma unroll
        for (int q = 0; q < kSweepRays; ++q) {
            iwl[q] = q == 0 ? make_wl_rcp(r[0].wl) : iwl[0];   // every phase update's divisor, 2 pi / wl
            gn[q] = (cptr<double>)(a.gn) + grp[q] * (4 * a.nsurf + 1);
        }
#pragma unroll
        for (int q = 0; q < kSweepRays; ++q) n_cur[q] = q == 0 ? mat_n(0, 0) : n_cur[0];
        trace_from(0);
#pragma unroll
        for (int q = 0; q < kSweepRays; ++q) reduce(r[q], tile[q] * kBlock + tid < a.gsize, grp[q], tile[q]);
    } else {
        const int32_t off = a.rows[2 * blockIdx.y], nb = a.rows[2 * blockIdx.y + 1];
        const int64_t t0 = blockIdx.x;
        const Ray<double> rg = gen(t0 * kBlock + tid, a.grp + 4 * int64_t(a.gidx[off]));
        wl0 = rg.wl;
        const int code0 = a.nsurf > 0 ? code_of(0) : -1;
        using std::integral_constant;
        // fn(kind, geo) on the first surface's code when it is a refracting Flat / Sphere; false otherwise
        auto on_first = [&](auto&& fn) {
            if (code0 == 3 * SPHERE + kGeoAxial) fn(integral_constant<int, SPHERE>(), integral_constant<int, kGeoAxial>());
            else if (code0 == 3 * SPHERE) fn(integral_constant<int, SPHERE>(), integral_constant<int, kGeoGeneral>());
            else if (code0 == 3 * FLAT + kGeoAxial) fn(integral_constant<int, FLAT>(), integral_constant<int, kGeoAxial>());
            else if (code0 == 3 * FLAT + kGeoXZ) fn(integral_constant<int, FLAT>(), integral_constant<int, kGeoXZ>());
            else if (code0 == 3 * FLAT) fn(integral_constant<int, FLAT>(), integral_constant<int, kGeoGeneral>());
            else return false;
            return true;
        };
        // the shared part of the first surface (surface_step_pair): a row that fails the front-side or on-surface
        // test stores a NaN position and c . d, so each refraction of it is all NaN (as the step's kill)
        const bool shared = on_first([&](auto kind, auto geo) {
            constexpr int K = decltype(kind)::value;
            constexpr int A = decltype(geo)::value;
            const DevSurface<double> base = load_surface<double>(surf);
            const Rcp<double> iwl0 = make_wl_rcp(rg.wl);     // (the phase, and with it n1 and iwl0, is not kept)
            double rxy0 = rg.x * rg.x + rg.y * rg.y;
            double Nx, Ny, Nz;
            Ray<double> ri;
            bool fwd = true;
            hit_and_normal<double, K, A>(base, rg, 1.0, iwl0, static_cast<GuardBranch*>(nullptr),
                                         K == SPHERE && A == kGeoAxial ? &rxy0 : nullptr, ri, Nx, Ny, Nz, &fwd);
            const bool front_ok = !front_side_fails<A, true>(rg, base) && fwd;
            constexpr int kBasis = K == FLAT ? A : kGeoGeneral;
            const SnellBasis<double> b = snell_basis<kBasis>(ri, Nx, Ny, Nz, static_cast<GuardBranch*>(nullptr));
            bool ok;
            if constexpr (K == SPHERE) ok = on_sphere<A == kGeoAxial>(ri, base, A == kGeoAxial ? &rxy0 : nullptr) && front_ok;
            else ok = on_flat<A>(ri, base) && front_ok;
            double px = ri.x, py = ri.y, pz = ri.z, cd = b.cd;
            if (!ok) px = py = pz = cd = qnan<double>();
            state[0][tid] = px; state[1][tid] = py; state[2][tid] = pz;
            state[3][tid] = Nx; state[4][tid] = Ny; state[5][tid] = Nz;
            state[6][tid] = b.cx; state[7][tid] = b.cy; state[8][tid] = b.cz;
            state[9][tid] = cd; state[10][tid] = b.nd;
        });
        if (!shared) {
            state[0][tid] = rg.x; state[1][tid] = rg.y; state[2][tid] = rg.z;
            state[3][tid] = rg.dx; state[4][tid] = rg.dy; state[5][tid] = rg.dz;
        }
        for (int p = 0; p < nb; p += kSweepRays) {
#pragma unroll
            for (int q = 0; q < kSweepRays; ++q) {
                grp[q] = a.gidx[off + p + q];
                tile[q] = t0;
                gn[q] = (cptr<double>)(a.gn) + grp[q] * (4 * a.nsurf + 1);
                r[q].ph = 0.0;
                r[q].wl = stored<TS>(a.grp[4 * grp[q] + 3]);
            }
            int s0 = 0;
            const bool first = on_first([&](auto kind, auto geo) {
                constexpr int kBasis = decltype(kind)::value == FLAT ? decltype(geo)::value : kGeoGeneral;
                Ray<double> ri;
                ri.x = state[0][tid]; ri.y = state[1][tid]; ri.z = state[2][tid];
                ri.dx = ri.dy = ri.dz = 0.0;
                ri.ph = 0.0;
                const double Nx = state[3][tid], Ny = state[4][tid], Nz = state[5][tid];
                SnellBasis<double> b;
                b.cx = state[6][tid]; b.cy = state[7][tid]; b.cz = state[8][tid];
                b.cd = state[9][tid]; b.nd = state[10][tid];
#pragma unroll
                for (int q = 0; q < kSweepRays; ++q) {
                    ri.wl = r[q].wl;
                    r[q] = snell_apply<kBasis, false>(ri, Nx, Ny, Nz, b, gn[q][a.nsurf + 1],
                                                        static_cast<GuardBranch*>(nullptr));
                }
            });
            if (first) {
                s0 = 1;
            } else {
#pragma unroll
                for (int q = 0; q < kSweepRays; ++q) {
                    r[q].x = state[0][tid]; r[q].y = state[1][tid]; r[q].z = state[2][tid];
                    r[q].dx = state[3][tid]; r[q].dy = state[4][tid]; r[q].dz = state[5][tid];
                }
            }
#pragma unroll
            for (int q = 0; q < kSweepRays; ++q) {
                iwl[q] = make_wl_rcp(r[q].wl);
                n_cur[q] = mat_n(q, s0);
            }
            trace_from(s0);
#pragma unroll
            for (int q = 0; q < kSweepRays; ++q) reduce(r[q], t0 * kBlock + tid < a.gsize, grp[q], t0);
        }
    }
}

// griddata(method='linear') on a regular grid + the pupil field of the PSF script (rtpb_grid_interpolate).
__global__ __launch_bounds__(kBlock) void grid_interp_kernel(rtpb_triangulation t, const double* __restrict__ xs,
                                                             int64_t nx, const double* __restrict__ ys, int64_t ny,
                                                             double radius, double* __restrict__ phase_out,
                                                             double* __restrict__ field_out) {
    const int64_t k = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (k >= nx * ny) return;
    const int64_t iy = k / nx, ix = k % nx;
    const double x = xs[ix], y = ys[iy];
    constexpr double eps = 100.0 * 2.220446049250313e-16;      // scipy qhull: 100 * DBL_EPSILON
    double phase = __builtin_nan("");
    const double fx = (x - t.x0) / t.cell_w, fy = (y - t.y0) / t.cell_h;
    if (fx >= 0.0 && fy >= 0.0 && fx < double(t.cells_x) && fy < double(t.cells_y)) {
        const int64_t cell = int64_t(fy) * t.cells_x + int64_t(fx);
        for (int32_t q = t.cell_start[cell]; q < t.cell_start[cell + 1]; ++q) {
            const int32_t s = t.cell_tris[q];
            const double* T = t.transform + 6 * int64_t(s);
            // scipy/spatial/_qhull.pyx _barycentric_inside / _barycentric_coordinates (ndim = 2)
            double c0 = 0.0;
            c0 += T[0] * (x - T[4]);
            c0 += T[1] * (y - T[5]);
            double c1 = 0.0;
            c1 += T[2] * (x - T[4]);
            c1 += T[3] * (y - T[5]);
            const double c2 = (1.0 - c0) - c1;
            if (!(-eps <= c0 && c0 <= 1.0 + eps) || !(-eps <= c1 && c1 <= 1.0 + eps) ||
                !(-eps <= c2 && c2 <= 1.0 + eps))
                continue;
            // scipy/interpolate/_interpnd.pyx LinearNDInterpolator._do_evaluate
            const int32_t* v = t.simplices + 3 * int64_t(s);
            double o = 0.0;
            o = o + c0 * t.values[v[0]];
            o = o + c1 * t.values[v[1]];
            o = o + c2 * t.values[v[2]];
            phase = o;
            break;
        }
    }
    if (phase_out) phase_out[k] = phase;
    if (field_out) {
        const bool off = sqrt(x * x + y * y) > radius || phase != phase;
        field_out[2 * k] = off ? 0.0 : cos(phase);
        field_out[2 * k + 1] = off ? 0.0 : sin(phase);
    }
}


}  // namespace

extern "C" {

int rtpb_intersect_rays(int32_t device, int32_t dtype, const void* ray1, int64_t n1, const void* ray2, int64_t n2,
                        void* pts_out, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad dtype");
    if (n1 < 0 || n2 < 0 || (n1 != n2 && n1 != 1 && n2 != 1))
        return fail(RTPB_E_INVALID, "ray1 and ray2 must be the same length");
    const int64_t n = std::max(n1, n2);
    if (n == 0) return RTPB_OK;
    if (!ray1 || !ray2 || !pts_out) return fail(RTPB_E_INVALID, "NULL pointer");
    IsectArgs a{ray1, ray2, pts_out, n, n1, n2};
    DeviceGuard g(device);
    const unsigned blocks = static_cast<unsigned>((n + kBlock - 1) / kBlock);
    if (dtype == RTPB_F64)
        hipLaunchKernelGGL(intersect_kernel<double>, dim3(blocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream), a);
    else
        hipLaunchKernelGGL(intersect_kernel<float>, dim3(blocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream), a);
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}

int rtpb_spot_stats(int32_t device, int32_t dtype, const void* plane, int64_t group_size, int64_t n_groups,
                    double* workspace, int64_t workspace_len, double* stats_out, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad dtype");
    if (group_size <= 0 || n_groups <= 0 || !plane || !stats_out || !workspace)
        return fail(RTPB_E_INVALID, "bad spot-stats arguments");
    const int64_t tiles = (group_size + kBlock - 1) / kBlock;
    if (workspace_len < n_groups * tiles * kStats)
        return fail(RTPB_E_INVALID, "workspace too small: need n_groups * ceil(group_size/256) * 7 doubles");
    if (tiles > 65535 * 16384ll || n_groups > 65535) return fail(RTPB_E_LIMIT, "too many groups");
    SpotArgs a{plane, workspace, stats_out, group_size, n_groups, tiles};
    DeviceGuard g(device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(n_groups));
    if (dtype == RTPB_F64) hipLaunchKernelGGL(spot_partial_kernel<double>, grid, dim3(kBlock), 0, st, a);
    else hipLaunchKernelGGL(spot_partial_kernel<float>, grid, dim3(kBlock), 0, st, a);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(spot_final_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(kBlock), 0, st, a);
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}

int rtpb_spot_sweep(const rtpb_plan* plan_c, int32_t device, int64_t n_groups, const double* group_params,
                    int64_t n_thetas, int64_t nphis, const double center_ray[3], const double ex[3],
                    const double ey[3], const double* theta_cos_sin, const double* phi_cos_sin, double* workspace,
                    int64_t workspace_len, double* stats_out, void* stream) {
    auto* plan = const_cast<rtpb_plan*>(plan_c);
    if (!plan) return fail(RTPB_E_INVALID, "plan is NULL");
    int rc = check_device(device);
    if (rc) return rc;
    if (n_groups <= 0 || n_thetas <= 0 || nphis <= 0 || !group_params || !center_ray || !ex || !ey ||
        !theta_cos_sin || !phi_cos_sin || !workspace || !stats_out)
        return fail(RTPB_E_INVALID, "bad spot-sweep arguments");
    const int64_t gsize = n_thetas * nphis;
    const int64_t tiles = (gsize + kBlock - 1) / kBlock;
    if (workspace_len < n_groups * tiles * kStats)
        return fail(RTPB_E_INVALID, "workspace too small: need n_groups * ceil(n_thetas*nphis/256) * 7 doubles");
    if (tiles > 0x7fffffffll || n_groups > 65535) return fail(RTPB_E_LIMIT, "too many groups or rays per group");
    DeviceGuard g(device);
    void* blob = nullptr;
    rc = plan_device_blob(plan, device, &blob);
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // one upload: trig tables, the per-group parameters, and (no POLY6 material) every material's n at
    // each group's wavelength -- material_n on the host, i.e. the kernel's own arithmetic (-ffp-contract=
    // off, IEEE division and sqrt), at the wavelength the kernel would see (rounded to the storage type)
    const bool pre_n = (plan->feat & 2) == 0;
    const size_t M = plan->mats.size();
    const size_t ntab = size_t(n_thetas + nphis);
    const size_t S = static_cast<size_t>(plan->nsurf);
    const size_t per_group = M + 3 * S;                 // n of every material, then n_s/n_s+1, 1/n_s+1, flags
    // block rows: groups of one field point in bundles of kSweepRays..kMaxBundle (multiples of kSweepRays; see
    // sweep_kernel), the rest single.
    // Bundles need the host-evaluated media (pre_n).
    std::vector<int32_t> bundles, rows, singles;
    {
        std::map<std::array<uint64_t, 3>, std::vector<int32_t>> by_point;   // field point (bit patterns) -> groups
        for (int64_t gi = 0; gi < n_groups; ++gi) {
            std::array<uint64_t, 3> key;
            std::memcpy(key.data(), group_params + 4 * gi, 3 * sizeof(double));
            if (pre_n) by_point[key].push_back(static_cast<int32_t>(gi));
            else singles.push_back(static_cast<int32_t>(gi));
        }
        for (const auto& kv : by_point) {
            const auto& gs = kv.second;
            size_t k = 0;
            while (gs.size() - k >= size_t(kSweepRays)) {
                const size_t left = gs.size() - k;
                const size_t nb = std::min<size_t>(kMaxBundle, left - left % kSweepRays);
                rows.push_back(static_cast<int32_t>(bundles.size()));
                rows.push_back(static_cast<int32_t>(nb));
                bundles.insert(bundles.end(), gs.begin() + k, gs.begin() + k + nb);
                k += nb;
            }
            for (; k < gs.size(); ++k) singles.push_back(gs[k]);
        }
        std::sort(singles.begin(), singles.end());
    }
    const size_t nidx = bundles.size() + singles.size() + rows.size();
    const size_t gn_bytes = pre_n ? size_t(n_groups) * per_group * sizeof(double) : 0;
    const size_t bytes = ntab * sizeof(double2) + size_t(4 * n_groups) * sizeof(double) + gn_bytes +
                         nidx * sizeof(int32_t);
    void* dbuf = nullptr;
    HIP_TRY(hipMallocAsync(&dbuf, bytes, st));
    PinnedStaging& g_pinned = pinned_staging();
    rc = g_pinned.reserve(bytes);
    if (rc) return rc;
    std::memcpy(g_pinned.buf, theta_cos_sin, size_t(2 * n_thetas) * sizeof(double));
    std::memcpy(g_pinned.buf + 2 * n_thetas, phi_cos_sin, size_t(2 * nphis) * sizeof(double));
    std::memcpy(g_pinned.buf + 2 * ntab, group_params, size_t(4 * n_groups) * sizeof(double));
    if (pre_n) {
        double* gn = g_pinned.buf + 2 * ntab + 4 * n_groups;
        std::vector<DevMaterial<double>> dm(M);
        for (size_t k = 0; k < M; ++k) dm[k] = device_material(*plan, k);
        for (int64_t gi = 0; gi < n_groups; ++gi) {
            const double w = group_params[4 * gi + 3];
            const double wl = plan->dtype == RTPB_F32 ? double(float(w)) : w;
            double* q = gn + gi * per_group;
            for (size_t k = 0; k < M; ++k) q[k] = material_n<double, false, true>(dm[k], wl, plan->table.data());
            for (size_t k = 0; k < S; ++k) {
                q[M + k] = q[k] / q[k + 1];
                q[M + S + k] = 1.0 / q[k + 1];
                q[M + 2 * S + k] = host_rcp_ok(q[k + 1]) ? 1.0 : 0.0;
            }
        }
    }
    const size_t idx_off = ntab * sizeof(double2) + size_t(4 * n_groups) * sizeof(double) + gn_bytes;
    int32_t* hidx = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(g_pinned.buf) + idx_off);
    std::copy(bundles.begin(), bundles.end(), hidx);
    std::copy(singles.begin(), singles.end(), hidx + bundles.size());
    std::copy(rows.begin(), rows.end(), hidx + bundles.size() + singles.size());
    rc = g_pinned.upload(dbuf, bytes, st);
    if (rc) return rc;
    SweepArgs a{};
    a.surf = static_cast<const DevSurface<double>*>(blob);
    a.mats = reinterpret_cast<const DevMaterial<double>*>(static_cast<char*>(blob) + plan->off_mats);
    a.table = reinterpret_cast<const double*>(static_cast<char*>(blob) + plan->off_table);
    a.tab = static_cast<const double2*>(dbuf);
    a.grp = reinterpret_cast<const double*>(static_cast<char*>(dbuf) + ntab * sizeof(double2));
    a.gn = a.grp + 4 * n_groups;
    const int32_t* didx = reinterpret_cast<const int32_t*>(static_cast<char*>(dbuf) + idx_off);
    a.partials = workspace;
    a.n_thetas = n_thetas;
    a.nphis = nphis;
    a.gsize = gsize;
    a.tiles = tiles;
    for (int j = 0; j < 3; ++j) {
        a.c[j] = center_ray[j]; a.ex[j] = ex[j]; a.ey[j] = ey[j];
    }
    a.nsurf = plan->nsurf;
    sweep_divisor(n_thetas, gsize, a.nt_mul, a.nt_shift);
    auto go = [&](auto tag) {
        using TS = decltype(tag);
        const int f = plan->feat & 3;                 // lens / POLY6 code (no pre_n: POLY6); tables always compiled in
        if (!rows.empty()) {
            SweepArgs ap = a;
            ap.gidx = didx;
            ap.rows = didx + bundles.size() + singles.size();
            const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(rows.size() / 2));
            if (f == 0) hipLaunchKernelGGL((sweep_kernel<TS, 16, true>), grid, dim3(kBlock), 0, st, ap);
            else hipLaunchKernelGGL((sweep_kernel<TS, 17, true>), grid, dim3(kBlock), 0, st, ap);
        }
        if (!singles.empty()) {
            SweepArgs as = a;
            as.gidx = didx + bundles.size();
            const dim3 grid(static_cast<unsigned>((tiles + kSweepRays - 1) / kSweepRays),
                            static_cast<unsigned>(singles.size()));
            if (pre_n && f == 0) hipLaunchKernelGGL((sweep_kernel<TS, 16, false>), grid, dim3(kBlock), 0, st, as);
            else if (pre_n) hipLaunchKernelGGL((sweep_kernel<TS, 17, false>), grid, dim3(kBlock), 0, st, as);
            else hipLaunchKernelGGL((sweep_kernel<TS, 3, false>), grid, dim3(kBlock), 0, st, as);   // POLY6 media
        }
    };
    if (plan->dtype == RTPB_F64) go(double{});
    else go(float{});
    HIP_TRY(hipGetLastError());
    SpotArgs sa{nullptr, workspace, stats_out, gsize, n_groups, tiles};
    hipLaunchKernelGGL(spot_final_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(kBlock), 0, st, sa);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipFreeAsync(dbuf, st));
    return RTPB_OK;
}

int rtpb_grid_interpolate(int32_t device, const rtpb_triangulation* tri, const double* xs, int64_t nx,
                          const double* ys, int64_t ny, double radius, double* phase_out, double* field_out,
                          void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (!tri || !xs || !ys || nx <= 0 || ny <= 0) return fail(RTPB_E_INVALID, "bad grid-interpolate arguments");
    if (tri->n_tri < 0 || (tri->n_tri > 0 && (!tri->transform || !tri->simplices || !tri->values)) ||
        tri->cells_x <= 0 || tri->cells_y <= 0 || !tri->cell_start || !tri->cell_tris || !(tri->cell_w > 0.0) ||
        !(tri->cell_h > 0.0))
        return fail(RTPB_E_INVALID, "bad triangulation descriptor");
    if (!phase_out && !field_out) return RTPB_OK;
    DeviceGuard g(device);
    const int64_t total = nx * ny;
    hipLaunchKernelGGL(grid_interp_kernel, dim3(static_cast<unsigned>((total + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, static_cast<hipStream_t>(stream), *tri, xs, nx, ys, ny, radius, phase_out, field_out);
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}

}  // extern "C"
