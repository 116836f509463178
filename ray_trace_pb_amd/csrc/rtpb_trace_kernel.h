// rtpb_trace_kernel.h -- the fused trace kernel (the hot path) and its launch dispatch, templated on
// the input element type TIN and the storage type TS.  Each rtpb_trace_<tin>_<ts>[_g1].hip translation unit
// instantiates launch_trace_group for one (TIN, TS) pair and one group of plan-feature variants, so the variants
// compile in parallel; the host side (rtpb_trace.hip) only sees launch_trace in rtpb_internal.h.
//
// plan (replacing System.ray_trace's surface loop RT:658-659 and the per-surface NumPy ufunc chains of
// RT:1160-1801), plus the host-buffer pipeline, tuning knobs and launch timing of the C ABI.
// Hot path: ONE kernel launch traces every ray through every surface of the system (replacing the
// Python surface loop RT:658-659 and the per-surface NumPy ufunc chains of RT:1160-1801).  One lane
// owns one ray for the whole system:
//   * the ray record (8 values) is read once from HBM (AOS: 16-byte vector loads; SOA: coalesced
//     per-field loads) and kept in VGPRs;
//   * surface and material descriptors are wave-uniform -- they are read through constant-address-
//     space pointers with uniform indices, i.e. scalar loads (s_load) into SGPRs, once per wave;
//   * n(lambda) of every material is evaluated once per ray (the reference re-evaluates it 3-4x per
//     surface, MAT:39-51 via RT:297/1213/1512) and carried across the surface loop;
//   * every requested history plane is written exactly once, at its final location -- no
//     O(S^2 N) re-copying of the history (RT:1229-1232);
//   * per-ray failures are NaN selects, never divergent early exits, so a wave stays converged.
// The surface loop is wave-uniform (same system for every lane), so its `kind` switches never diverge.
//
// Precision: arithmetic is ALWAYS float64 in registers (the reference's numerics); the storage type TS
// of the ray buffers is float64 or float32.  float32 storage halves the HBM bytes (the bound) while the
// values stay the correctly rounded float64 results: a float32 trace equals the float64 reference on the
// float32-rounded input, rounded once on store.
//
// Memory roofline: per ray the kernel moves 8w bytes in and 8w bytes per stored plane out
// (w = sizeof(TS)); see DESIGN.md for the algorithmic-byte accounting used by bench.py.

#pragma once

#include "rtpb_internal.h"

namespace rtpbi {


// Workgroup size per variant: the LDS-staged AoS kernels run one wave per workgroup (see kTraceBlock);
// the direct-store variants (SoA output, unstaged AoS) keep four-wave workgroups, which measured faster
// for their strided stores (C5 SoA: 0.53 vs 0.69 ms).
constexpr int trace_block(int out_layout, int store) {
    return (out_layout == RTPB_AOS && (store & 1)) ? kTraceBlock : 256;
}

// The fused multi-surface trace: one lane = one ray through all surfaces (float64 arithmetic, TS
// storage).  STORE: bit 0 = LDS-staged AOS stores (OUT_LAYOUT == AOS only), bit 1 = non-temporal global
// stores for the staged tiles, bit 2 = LDS-staged AOS input loads, bit 3 = final plane only.
// FEAT: bit 0 = PerfectLens code, bit 1 = RTPB_POLY6 code compiled in, bit 2 = TABLE materials looked up
// in an LDS copy of the plan's table (dynamic LDS, copied at launch), bit 3 = TABLE materials looked up
// in global memory.  Leaving out what a plan does not use lowers register pressure (round 2's f64 staged kernels:
// 92 VGPRs without the PerfectLens code, 100 with both), 10-15 % faster when compute-bound, and without a global
// table lookup the surface loop never waits on the vmcnt counter, which on gfx950 would also wait for
// every history store in flight (see kLdsTablePairs).  rtpb_plan::feat picks the variant.
template <typename TIN, typename TS, int IN_LAYOUT, int OUT_LAYOUT, int STORE, int WPE, int FEAT>
__global__ __launch_bounds__(trace_block(OUT_LAYOUT, STORE)) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
void trace_kernel(TraceArgs<TIN, TS> a) {
    constexpr int kB = trace_block(OUT_LAYOUT, STORE);
    using T = double;
    constexpr bool kStaged = (STORE & 1) && OUT_LAYOUT == RTPB_AOS;
    constexpr bool kNT = (STORE & 2) != 0;
    // STORE bit 4: float32 records flushed by a register exchange instead of the LDS tiles (xchg_flush)
    constexpr bool kXchg = (STORE & 16) != 0;
    static_assert(!kXchg || (kStaged && sizeof(TS) == 4 && kB == 64), "exchange flush: staged float32 AOS");
    // STORE bit 3: only the final plane is stored (planes='final'): no per-surface store logic, one
    // LDS tile, fewer live registers (the C5 / spot-diagram and focus-finding mode)
    constexpr bool kFinal = (STORE & 8) != 0;
    constexpr bool kLens = (FEAT & 1) != 0, kPoly = (FEAT & 2) != 0;
    constexpr int kKinds = (FEAT & 32) != 0 ? kKindsLensFlat : kKindsAll;    // rtpb_plan::feat bit 32
    constexpr bool kTabLds = (FEAT & 12) == 4, kTabGlobal = (FEAT & 8) != 0, kIdx = (FEAT & 16) != 0;
    extern __shared__ double lds_table[];                // FEAT bit 2: the plan's (wavelength, n) pairs;
                                                         // FEAT bit 4: the indexed-material table
    if constexpr (kTabLds || kIdx) {
        // before any wave can leave: the unstaged variants run four-wave workgroups and need the barrier
        const int cnt = kIdx ? a.nkeys * (2 * a.nsurf + 2) : 2 * a.ntable;
        const double* src = kIdx ? a.itab : a.table;
        for (int k = threadIdx.x; k < cnt; k += kB) lds_table[k] = src[k];
        if constexpr (kB > 64) __syncthreads();
    }
    // per wave: "at" and "after" tiles of 64 records (4 KiB f64, 2 KiB f32: the LDS budget allows 5 f64 /
    // 10 f32 waves per SIMD in the all-planes mode, so registers set the f32 occupancy)
    __shared__ uint4 tiles[kB / 64][kFinal ? 1 : 2][kTileBytes / 16 * sizeof(TS) / 8];
    const int lane = threadIdx.x & 63;
    // one block of kB rays per workgroup (blocks go round-robin over the XCDs: measured faster than
    // XCD-contiguous block ranges).  The body is a lambda of the block index; called once.
    auto body = [&](const int64_t blk) {
    const int64_t i = kXchg ? blk * kB + xchg_ray(lane) : blk * kB + threadIdx.x;
    const int64_t ray0 = kXchg ? blk * kB
                               : static_cast<int64_t>(uniform_u64(static_cast<uint64_t>(i - lane)));  // first ray of this wave
    if (ray0 >= a.n) return;                             // wave-uniform exit
    const bool valid = i < a.n;
    uint4* tile_a = tiles[threadIdx.x >> 6][0];
    uint4* tile_b = tiles[threadIdx.x >> 6][kFinal ? 0 : 1];
    Ray<T> r;
    // staged input loads use the output tile, so they need the input records to be TS-sized
    if constexpr (kStaged && IN_LAYOUT == RTPB_AOS && (STORE & 4) && std::is_same<TIN, TS>::value)
        r = tile_load<TS>(tile_b, a.in, ray0, a.n, lane);
    else r = load_ray<TIN, IN_LAYOUT>(a.in, valid ? i : a.n - 1, a.in_fs);
    const T wl0 = r.wl;
    const Rcp<T> iwl = make_wl_rcp(wl0);                 // shared divisor of every phase update, 2 pi / wl
    TS* __restrict__ out = a.out;
    const cptr<DevSurface<T>> surf = (cptr<DevSurface<T>>)(a.surf);
    const cptr<DevMaterial<T>> mats = (cptr<DevMaterial<T>>)(a.mats);
    const cptr<T> table = (cptr<T>)(a.table);
    // indexed materials: the ray's key once (-1 = wavelength not among the plan's keys: every material
    // is then evaluated as without the index, TABLE materials giving NaN as a table miss does)
    const int widx = kIdx ? key_index(lds_table, a.nkeys, wl0) : -1;
    if constexpr (kIdx || kTabLds || kTabGlobal) {
        // rtpb_trace_checked: flag rays whose wavelength is not a table key (wave-uniform pointer test;
        // every flagging lane stores the same value, so no atomic is needed)
        if (a.miss != nullptr) {
            bool miss = false;
            if constexpr (kIdx) {
                miss = widx < 0;
            } else {
                for (int k = 0; k <= a.nsurf; ++k) {
                    const DevMaterial<T> m = load_material<T>(mats + k);
                    if (m.kind == TABLE)
                        miss = miss || !(kTabLds ? table_has_key(m, wl0, static_cast<const double*>(lds_table))
                                                 : table_has_key(m, wl0, table));
                }
            }
            if (valid && miss) a.miss[0] = 1;
        }
    }
    // every lane of the wave has its key: the surfaces' Snell ratios come from the table too (uniform test)
    const bool all_idx = kIdx && __builtin_amdgcn_ballot_w64(widx < 0) == 0;
    // every lane's Vacuum index is exactly 1 (wavelength squared finite and nonzero, MAT:54-56): the host's
    // ratios of Constant / Vacuum boundaries hold for the whole wave (uniform test)
    const T w2 = wl0 * wl0;
    const bool vac_one = __builtin_amdgcn_ballot_w64(!(w2 != T(0) && w2 - w2 == T(0))) == 0;
    auto surface = [&](int s) -> DevSurface<T> {
        DevSurface<T> d = load_surface<T>(surf + s);
        if ((d.rcp_ok & 16) && vac_one) d.rcp_ok |= 4 | ((d.rcp_ok & 32) ? 8 : 0);
        if ((d.rcp_ok & kLensUniVac) && vac_one) d.rcp_ok |= kLensUni;
        if constexpr (kIdx) {
            if (all_idx && !(d.rcp_ok & 4)) {
                d.nr = lds_table[a.nkeys * (a.nsurf + 2 + s) + widx];
                d.rcp_ok |= 4;
            }
        }
        return d;
    };
    auto mat_n = [&](cptr<DevMaterial<T>> mp) -> T {
        if constexpr (kIdx) {
            if (widx >= 0) return lds_table[a.nkeys * (1 + static_cast<int>(mp - mats)) + widx];
            return material_n<T, false, false>(load_material<T>(mp), wl0, table);
        } else if constexpr (kTabLds) {
            return material_n<T, kPoly, true>(load_material<T>(mp), wl0, lds_table);
        } else {
            return material_n<T, kPoly, kTabGlobal>(load_material<T>(mp), wl0, table);
        }
    };
    if constexpr (kFinal) {
        T n_cur = mat_n(mats);
        // two surfaces per iteration, the second writing straight into the loop-carried ray: the register
        // allocator cannot coalesce a step's output with the ray it read across the kind switch (a copy of all
        // eight values per surface otherwise)
        for (int s = 0; s < a.nsurf; s += 2) {
            const T n_mid = mat_n(mats + s + 1);
            Ray<T> mid;
            propagate_surface_emit<T, kLens, kNoAt, kKinds>(surface(s), r, n_cur, n_mid, iwl, [](const Ray<T>&) {}, mid);
            if (s + 1 < a.nsurf) {
                const T n_next = mat_n(mats + s + 2);
                propagate_surface_emit<T, kLens, kNoAt, kKinds>(surface(s + 1), mid, n_mid, n_next, iwl, [](const Ray<T>&) {},
                                                        r);
                n_cur = n_next;
            } else {
                r = mid;
                n_cur = n_mid;
            }
        }
        if constexpr (kXchg) {
            xchg_flush<kNT>(out, ray0, a.n, lane, r);
        } else if constexpr (kStaged) {
            tile_write<TS>(tile_b, lane, r);
            lds_wait();
            tile_flush<TS, kNT>(tile_b, out, ray0, a.n, lane);
        } else if (valid) {
            store_ray<TS, OUT_LAYOUT>(out, i, a.out_fs, r);
        }
        return;
    }
    int64_t slot_off = 0;
    if (a.mask_lo & 1ull) {
        if constexpr (kXchg) {
            xchg_flush<kNT>(out, ray0, a.n, lane, r);
        } else if constexpr (kStaged) {
            tile_write<TS>(tile_a, lane, r);
            lds_wait();
            tile_flush<TS, kNT>(tile_a, out, ray0, a.n, lane);
        } else if (valid) {
            store_ray<TS, OUT_LAYOUT>(out, i, a.out_fs, r);
        }
        slot_off += a.out_ps;
    }
    // one surface with its planes: `in` -> `out` (two per iteration below, so the second writes straight into the
    // loop-carried ray -- no per-surface copy of the ray across the kind switch)
    auto one = [&](int s, const Ray<T>& in, T n_in, Ray<T>& res, T& n_res) {
        const T n_next = mat_n(mats + s + 1);
        const int p = 2 * s + 1;
        const bool st_at = plane_bit(a.mask_lo, a.mask_hi, p);          // wave-uniform
        const bool st_after = plane_bit(a.mask_lo, a.mask_hi, p + 1);
        const int64_t off_at = slot_off;
        slot_off += st_at ? a.out_ps : 0;
        const int64_t off_after = slot_off;
        slot_off += st_after ? a.out_ps : 0;
        // the "at" plane goes to its LDS tile (or straight out) as soon as it is final
        auto emit_at = [&](const Ray<T>& at) {
            if constexpr (kXchg) {
                if (st_at) xchg_flush<kNT>(out + off_at, ray0, a.n, lane, at);
            } else if constexpr (kStaged) {
                if (st_at) tile_write<TS>(tile_a, lane, at);
            } else {
                if (valid && st_at) store_ray<TS, OUT_LAYOUT>(out + off_at, i, a.out_fs, at);
            }
        };
        propagate_surface_emit<T, kLens, 0, kKinds>(surface(s), in, n_in, n_next, iwl, emit_at, res);
        if constexpr (kXchg) {
            if (st_after) xchg_flush<kNT>(out + off_after, ray0, a.n, lane, res);
        } else if constexpr (kStaged) {
            // both planes of the surface share one LDS round trip
            if (st_after) tile_write<TS>(tile_b, lane, res);
            if (st_at || st_after) lds_wait();
            if (st_at) tile_flush<TS, kNT>(tile_a, out + off_at, ray0, a.n, lane);
            if (st_after) tile_flush<TS, kNT>(tile_b, out + off_after, ray0, a.n, lane);
        } else if (valid) {
            if (st_after) store_ray<TS, OUT_LAYOUT>(out + off_after, i, a.out_fs, res);
        }
        n_res = n_next;
    };
    T n_cur = mat_n(mats);
    for (int s = 0; s < a.nsurf; s += 2) {
        Ray<T> mid;
        T n_mid;
        one(s, r, n_cur, mid, n_mid);
        if (s + 1 < a.nsurf) {
            one(s + 1, mid, n_mid, r, n_cur);
        } else {
            r = mid;
            n_cur = n_mid;
        }
    }
    };
    body(static_cast<int64_t>(blockIdx.x));
}



template <typename TI, typename T, int IL, int OL, int ST, int W, int FEAT>
hipError_t launch_w(const TraceArgs<TI, T>& a, hipStream_t st) {
    constexpr int kB = trace_block(OL, ST);
    const int64_t blocks = (a.n + kB - 1) / kB;
    const size_t lds = (FEAT & 16)        ? static_cast<size_t>(a.nkeys) * (2 * a.nsurf + 2) * sizeof(double)
                       : (FEAT & 12) == 4 ? static_cast<size_t>(a.ntable) * 2 * sizeof(double) : 0;
    hipLaunchKernelGGL((trace_kernel<TI, T, IL, OL, ST, W, FEAT>), dim3(static_cast<unsigned>(blocks)), dim3(kB), lds,
                       st, a);
    return hipGetLastError();
}

template <typename TI, typename T, int IL, int OL, int ST, int GROUP>
hipError_t launch_one(const TraceArgs<TI, T>& a, int feat, hipStream_t st) {
    // float64 final-plane-only kernels (compute-bound: the C5 / focus-finding mode) are held to >= 6
    // waves per SIMD (<= 80 VGPRs, no spill; 7 and 8 measured slower); everything else keeps the
    // compiler's choice (the history kernels are bound by their LDS tiles and store stream: 6-8 waves
    // measured no faster; the float32 final-only variants would spill)
#define RTPB_WPE(F) (((ST & 8) && sizeof(T) == 8 && (F) != 15) ? 6 : 1)
    if constexpr (GROUP == 0) {
        switch (feat) {
        case 0: return launch_w<TI, T, IL, OL, ST, RTPB_WPE(0), 0>(a, st);
        case 1: return launch_w<TI, T, IL, OL, ST, RTPB_WPE(1), 1>(a, st);
        case 4: return launch_w<TI, T, IL, OL, ST, RTPB_WPE(4), 4>(a, st);
        case 5: return launch_w<TI, T, IL, OL, ST, RTPB_WPE(5), 5>(a, st);
        case 33: return launch_w<TI, T, IL, OL, ST, RTPB_WPE(33), 33>(a, st);
        default: return hipErrorInvalidValue;                                // another group's feature set
        }
    } else {
        switch (feat) {
        case 16: return launch_w<TI, T, IL, OL, ST, RTPB_WPE(16), 16>(a, st);
        case 17: return launch_w<TI, T, IL, OL, ST, RTPB_WPE(17), 17>(a, st);
        default: return launch_w<TI, T, IL, OL, ST, RTPB_WPE(15), 15>(a, st);   // POLY6 or a large table: everything
        }
    }
#undef RTPB_WPE
}

template <typename TI, typename T, int G>
hipError_t launch_trace_group(const TraceArgs<TI, T>& a, int il, int ol, int feat, hipStream_t st) {
    const int staging = g_aos_staging.load();
    const bool staged = staging != 0;
    const bool nt = g_nt_stores.load() != 0;
    // aos_staging 2: float32 storage flushed by register exchange (STORE bit 4) instead of LDS tiles
    constexpr bool kF32 = sizeof(T) == 4;
    const bool xchg = kF32 && staging == 2 && nt;
    const int last = 2 * a.nsurf;                       // planes='final': only the last plane stored
    const bool final_only = a.nsurf > 0 && (last < 64 ? (a.mask_lo == (1ull << last) && a.mask_hi == 0)
                                                      : (a.mask_lo == 0 && a.mask_hi == (1ull << (last - 64))));
    if (final_only && ol == RTPB_AOS && il == RTPB_AOS && staged && nt && !g_stage_input.load())
    {
        if constexpr (kF32) {
            if (xchg) return launch_one<TI, T, RTPB_AOS, RTPB_AOS, 27, G>(a, feat, st);
        }
        return launch_one<TI, T, RTPB_AOS, RTPB_AOS, 11, G>(a, feat, st);
    }
    if constexpr (!std::is_same<TI, T>::value) {
        // input and storage types differ: AOS input only (rtpb_trace checks), no staged-input variant
        if (ol == RTPB_SOA) return launch_one<TI, T, RTPB_AOS, RTPB_SOA, 0, G>(a, feat, st);
        if (!staged) return launch_one<TI, T, RTPB_AOS, RTPB_AOS, 0, G>(a, feat, st);
        if constexpr (kF32) {
            if (xchg) return launch_one<TI, T, RTPB_AOS, RTPB_AOS, 19, G>(a, feat, st);
        }
        return nt ? launch_one<TI, T, RTPB_AOS, RTPB_AOS, 3, G>(a, feat, st) : launch_one<TI, T, RTPB_AOS, RTPB_AOS, 1, G>(a, feat, st);
    }
    if (ol == RTPB_AOS) {
        if (!staged)
            return il == RTPB_AOS ? launch_one<TI, T, RTPB_AOS, RTPB_AOS, 0, G>(a, feat, st) : launch_one<TI, T, RTPB_SOA, RTPB_AOS, 0, G>(a, feat, st);
        if (nt && il == RTPB_AOS && g_stage_input.load()) return launch_one<TI, T, RTPB_AOS, RTPB_AOS, 7, G>(a, feat, st);
        if constexpr (kF32) {
            if (xchg && il == RTPB_AOS) return launch_one<TI, T, RTPB_AOS, RTPB_AOS, 19, G>(a, feat, st);
        }
        if (nt)
            return il == RTPB_AOS ? launch_one<TI, T, RTPB_AOS, RTPB_AOS, 3, G>(a, feat, st) : launch_one<TI, T, RTPB_SOA, RTPB_AOS, 3, G>(a, feat, st);
        return il == RTPB_AOS ? launch_one<TI, T, RTPB_AOS, RTPB_AOS, 1, G>(a, feat, st) : launch_one<TI, T, RTPB_SOA, RTPB_AOS, 1, G>(a, feat, st);
    }
    if (il == RTPB_AOS) return launch_one<TI, T, RTPB_AOS, RTPB_SOA, 0, G>(a, feat, st);
    return launch_one<TI, T, RTPB_SOA, RTPB_SOA, 0, G>(a, feat, st);
}


}  // namespace rtpbi
