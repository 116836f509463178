"""Named experiment variants of librtpb.so, built from a scratch copy of the sources with the source edits
defined here, so each experiment is reviewable and never touches the shipped code.  (The round-2
experiment switches -- RTPB_EXP_XCD_REMAP, PERSIST, STAGGER, ... -- are kept as a patch against the round-2
sources: profiles/r02/experiments/experiments_round2.patch.)

    python tools/exp_variants.py NAME [NAME ...]      # -> ray_trace_pb_amd/exp_<NAME>.so
    python tools/exp_variants.py --list

Variants that drop work are NOT bit-exact (ab_variants.py skips the output comparison for names that
contain "exp_no").
"""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ray_trace_pb_amd import _build  # noqa: E402

EXP_PATCH = os.path.join(ROOT, "profiles", "r02", "experiments", "experiments_round2.patch")

# name -> (use experiments.patch, -D flags, [(file, old, new)])
VARIANTS = {
    # the memory path alone: the surface arithmetic replaced by a copy (same loads, tiles and stores)
    "nocomp": (False, [], [(
        "rtpb_trace_kernel.h",
        "        propagate_surface_emit<T, kLens>(surface(s), r, n_cur, n_next, iwl, emit_at, after);",
        "        after = r; after.ph = r.ph + n_next + n_cur; emit_at(r);")]),
    # the compute side alone: LDS staging kept, global history stores dropped (the tile reads are kept
    # alive), i.e. what the kernel costs without the HBM write stream
    "nostore": (False, [], [(
        "rtpb_internal.h",
        "            __builtin_amdgcn_raw_buffer_store_b128(t[4 * rr + (pp ^ ((rr >> 1) & 3))], rsrc, c * 16, 0, kAux);",
        "            { v4u v_ = t[4 * rr + (pp ^ ((rr >> 1) & 3))]; asm volatile(\"\" :: \"v\"(v_)); (void)rsrc; }"), (
        "rtpb_internal.h",
        "            __builtin_amdgcn_raw_buffer_store_b128(t[2 * rr + (pp ^ ((rr >> 2) & 1))], rsrc, c * 16, 0, kAux);",
        "            { v4u v_ = t[2 * rr + (pp ^ ((rr >> 2) & 1))]; asm volatile(\"\" :: \"v\"(v_)); (void)rsrc; }")]),
    # input records read from a 1M-ray (64 MB) window that stays cache-resident: the real arithmetic on
    # real rays (repeated), all outputs written, no HBM input stream
    "l2input": (False, [], [(
        "rtpb_trace_kernel.h",
        "    else r = load_ray<TIN, IN_LAYOUT>(a.in, valid ? i : a.n - 1, a.in_fs);",
        "    else r = load_ray<TIN, IN_LAYOUT>(a.in, (valid ? i : a.n - 1) & ((1 << 20) - 1), a.in_fs);")]),
    # float64 input records of a float32 history read through the wave's two float32 tiles (4 KiB: one
    # coalesced 1 KiB load per instruction, then each lane reads its record from LDS) instead of four
    # 16-byte loads per lane at a 64-byte lane stride
    "stagein": (False, [], [(
        "rtpb_trace_kernel.h",
        "    else r = load_ray<TIN, IN_LAYOUT>(a.in, valid ? i : a.n - 1, a.in_fs);",
        "    else if constexpr (kStaged && !kFinal && !kXchg && IN_LAYOUT == RTPB_AOS && sizeof(TIN) == 8 &&\n"
        "                       sizeof(TS) == 4)\n"
        "        r = tile_load<TIN>(tile_a, a.in, ray0, a.n, lane);\n"
        "    else r = load_ray<TIN, IN_LAYOUT>(a.in, valid ? i : a.n - 1, a.in_fs);")]),
    # history kernels allowed more registers: at most 5 / 4 waves per SIMD (the scheduler's occupancy target)
    "wpemax5": (False, [], [(
        "rtpb_trace_kernel.h",
        "__attribute__((amdgpu_waves_per_eu(WPE, 8)))",
        "__attribute__((amdgpu_waves_per_eu(WPE, (STORE & 8) ? 8 : 5)))")]),
    "wpemax4": (False, [], [(
        "rtpb_trace_kernel.h",
        "__attribute__((amdgpu_waves_per_eu(WPE, 8)))",
        "__attribute__((amdgpu_waves_per_eu(WPE, (STORE & 8) ? 8 : 4)))")]),
    # float32 history kernels held to >= 6 waves per SIMD (<= 80 VGPRs)
    "wpe6hist": (False, [], [(
        "rtpb_trace_kernel.h",
        "#define RTPB_WPE(F) (((ST & 8) && sizeof(T) == 8 && (F) != 15) ? 6 : 1)",
        "#define RTPB_WPE(F) ((((ST & 8) && sizeof(T) == 8) || (!(ST & 8) && sizeof(T) == 4)) && (F) != 15 ? 6 : 1)")]),
    # round-3 math changes, one at a time reverted (bit-identical variants)
    "oldchk": (False, [], [(
        "rtpb_math.h",
        "    return static_cast<uint32_t>(__builtin_amdgcn_frexp_exp(b) + 119) <= 239u;",
        "    const uint32_t h2 = static_cast<uint32_t>(__double2hiint(b)) << 1;\n"
        "    return h2 - (903u << 21) < (240u << 21) || __builtin_amdgcn_class(b, 0x267);"), (
        "rtpb_math.h",
        "    return static_cast<uint32_t>(__builtin_amdgcn_frexp_exp(a) + 799) <= 1399u;",
        "    const uint32_t h2 = static_cast<uint32_t>(__double2hiint(a)) << 1;\n"
        "    return h2 - (223u << 21) < (1400u << 21) || __builtin_amdgcn_class(a, 0x267);")]),
    # ray blocks in a permuted order (groups of G consecutive blocks, the group order scattered by an odd
    # multiplier modulo the next power of two, cycle-walked into range): concurrently running waves write
    # each history plane at scattered offsets instead of one advancing window per plane
    **{f"perm{G}": (False, [], [(
        "rtpb_trace_kernel.h",
        "    body(static_cast<int64_t>(blockIdx.x));",
        "    {\n"
        f"        constexpr int64_t G = {G};\n"
        "        const int64_t ng = static_cast<int64_t>(gridDim.x) / G;\n"
        "        int64_t b = blockIdx.x;\n"
        "        const int64_t gi = b / G;\n"
        "        if (gi < ng) {\n"
        "            uint64_t K = 1;\n"
        "            while (K < static_cast<uint64_t>(ng)) K <<= 1;\n"
        "            uint64_t y = static_cast<uint64_t>(gi);\n"
        "            do { y = (y * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) & (K - 1); }\n"
        "            while (y >= static_cast<uint64_t>(ng));\n"
        "            b = static_cast<int64_t>(y) * G + (b % G);\n"
        "        }\n"
        "        body(b);\n"
        "    }")]) for G in (1, 16, 256)},
    # cache policy of the history stores (gfx950 cpol: sc0 = 1, nt = 2, sc1 = 16; shipped: nt | sc1)
    **{f"pol{v}": (False, [], [(
        "rtpb_internal.h", "constexpr int kAux = NT ? (2 | 16) : 0;", f"constexpr int kAux = NT ? {v} : 0;")])
       for v in (2, 3, 19, 17)},
    "noratio": (False, [], [(
        "rtpb_math.h",
        "            after = snell(ri, Nx, Ny, Nz, (s.rcp_ok & 4) ? s.nr : n1 / n2, g);",
        "            after = snell(ri, Nx, Ny, Nz, n1 / n2, g);")]),
}


def build(name):
    use_patch, flags, edits = VARIANTS[name]
    out = os.path.join(ROOT, "ray_trace_pb_amd", f"exp_{name}.so")
    with tempfile.TemporaryDirectory() as tmp:
        csrc = os.path.join(tmp, "ray_trace_pb_amd", "csrc")
        shutil.copytree(_build.CSRC, csrc, ignore=shutil.ignore_patterns("_obj"))
        if use_patch:
            subprocess.run(["patch", "-p1", "-s", "-d", tmp, "-i", EXP_PATCH], check=True)
        for fname, old, new in edits:
            p = os.path.join(csrc, fname)
            src = open(p).read()
            if old not in src:
                raise SystemExit(f"{name}: edit target not found in {fname}: {old[:80]}")
            open(p, "w").write(src.replace(old, new))
        _build.build(force=True, verbose=False, extra_flags=flags, out=out, csrc=csrc)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*")
    ap.add_argument("--list", action="store_true")
    args = ap.parse_args()
    if args.list:
        for k in VARIANTS:
            print(k)
        return
    for n in args.names:
        print(build(n), flush=True)


if __name__ == "__main__":
    main()
