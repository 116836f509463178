/*
 * rtpb.h -- C ABI of the MI355X-native sequential ray tracer (ray_trace_pb_amd).
 *
 * This is the drop-in boundary for the reference's hot path, QI2lab/ray_trace_pb @ 2024_10_08:
 *
 *   src/raytrace/raytrace.py:658-659  (System.ray_trace)
 *       for ii in range(len(self.surfaces)):
 *           rays = self.surfaces[ii].propagate(rays, materials[ii], materials[ii + 1])
 *
 * One rtpb_trace() call replaces that whole loop: every Surface.propagate of the system
 * (RefractingSurface RT:1160-1234, ReflectingSurface RT:1238-1303, PerfectLens RT:1601-1801 with
 * FlatSurface RT:1306-1347, PlaneMirror RT:1377-1412, SphericalSurface RT:1435-1535), every
 * propagate_ray2plane (RT:241-306) and every Material.n (materials.py:39-144) runs fused in one HIP
 * kernel per launch on gfx950 (Sellmeier / Constant n(lambda) evaluated in the kernel; other
 * materials looked up in (wavelength, n) tables the caller evaluated with the material's own code).  The history the reference builds with concatenate (RT:1229-1232) is
 * written plane by plane, straight to its final place in the caller's output buffer.
 *
 * Conventions
 *   - Plain C types only.  All ray buffers are caller-owned; the library never frees or retains them.
 *   - A ray is 8 values (x, y, z, dx, dy, dz, phase, wavelength) -- RT:1-13, RT:85-94.  Layout AOS
 *     stores a plane as [ray][8] (the reference's (P, N, 8) C order); layout SOA stores it as [8][ray].
 *   - History plane p: p = 0 is the input plane, p = 2i+1 the rays AT surface i, p = 2i+2 the rays
 *     AFTER surface i (RT:1229-1232, RT:1799).  `plane_mask` bit p selects which planes are stored;
 *     selected planes are packed in increasing p order into consecutive output slots.
 *   - Per-ray failures are not errors: they are NaN exactly as in the reference (miss RT:1506-1509,
 *     back-facing RT:1190-1192, TIR RT:1221, aperture RT:1225-1226/1293-1294, NA RT:1757-1760,
 *     backward RT:303-304/1401).
 *   - Every function returns RTPB_OK (0) or a negative RTPB_E_* code; rtpb_last_error() returns the
 *     message of the calling thread's last failure.  No C++ exception crosses the ABI.
 *   - Thread-safety: plans are immutable after creation and may be used from several threads at
 *     once; each (device, stream) pair must be driven by one thread at a time.
 */
#ifndef RTPB_H
#define RTPB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTPB_ABI_VERSION 9   /* 2: + *_tables generators, surface-hook kernels, sorted-table lookup
                                3: input element type separate from the storage type (in_dtype)
                                4: + rtpb_trace_checked (table-miss flag)
                                5: + rtpb_buffer_alloc / _free / _dlpack (placement-robust history buffers)
                                6: stream-ordered history buffers: rtpb_buffer_alloc takes the stream,
                                   + rtpb_buffer_record_stream / _held / _dlpack_discard
                                7: + rtpb_torch_alloc / rtpb_torch_free (torch MemPool segments),
                                   rtpb_buffer_stats; releasing a mapping synchronises the device;
                                   + rtpb_ray_fan_tables_wl / rtpb_collimated_rays_tables_wl (per-ray
                                   wavelengths)
                                8: + rtpb_trace_f64 / rtpb_trace_f32 (one-shot calls),
                                   rtpb_oneshot_plans / rtpb_oneshot_clear; freeing a library buffer
                                   never synchronises the device (retired mappings are released by the
                                   next allocation that maps new memory, or by rtpb_buffer_trim)
                                9: + rtpb_trace_packed (rtpb_trace_checked's arguments in one struct) */

/* ---- error codes ---------------------------------------------------------------------------- */
#define RTPB_OK 0
#define RTPB_E_INVALID (-1)   /* bad argument (kind, size, pointer, mask) */
#define RTPB_E_HIP (-2)       /* HIP runtime error */
#define RTPB_E_NODEV (-3)     /* no GPU / device index out of range */
#define RTPB_E_LIMIT (-4)     /* a compiled-in limit was exceeded (e.g. > RTPB_MAX_SURFACES) */

/* ---- enums ---------------------------------------------------------------------------------- */
/* surface kinds (reference classes) */
#define RTPB_FLAT 0          /* FlatSurface      RT:1306-1347 (refracting)          */
#define RTPB_SPHERE 1        /* SphericalSurface RT:1435-1535 (refracting)          */
#define RTPB_PLANE_MIRROR 2  /* PlaneMirror      RT:1377-1412 (reflecting)          */
#define RTPB_PERFECT_LENS 3  /* PerfectLens      RT:1558-1801 (ideal-lens mapping)  */

/* material kinds (Material.n overrides) */
#define RTPB_CONSTANT 0      /* Constant  MAT:59-79:  n = c[0]                                   */
#define RTPB_SELLMEIER 1     /* Material  MAT:39-51:  c = {b1,b2,b3,c1,c2,c3}; Vacuum = zeros    */
#define RTPB_POLY6 2         /* Ebaf11    MAT:128-144: c = {p0..p5}, n^2 = p0+p1 w^2+p2 w^-2+...
                                evaluated on the device with the device pow(): within 1 ulp of the
                                host's, but NumPy's SIMD power differs from libm pow on ~5 % of
                                inputs, so bit-exact callers lower Ebaf11 as RTPB_TABLE instead */
#define RTPB_TABLE 3         /* n looked up by exact wavelength match in a (wavelength, n) table
                                evaluated on the host by the material's own n() (user subclasses;
                                the Python front end also lowers Ebaf11 this way, see POLY6) */

/* data types and layouts */
#define RTPB_F64 0
#define RTPB_F32 1
#define RTPB_AOS 0
#define RTPB_SOA 1

/* surface-hook interaction modes (rtpb_interact) */
#define RTPB_REFRACT 0
#define RTPB_REFLECT 1

#define RTPB_MAX_SURFACES 63     /* history planes 0..2S must fit the 128-bit plane mask */
#define RTPB_MAX_TABLE (1 << 22) /* total (wavelength, n) entries over all TABLE materials */

/* ---- descriptors ---------------------------------------------------------------------------- */
typedef struct rtpb_surface {
    int32_t kind;           /* RTPB_FLAT ... */
    int32_t reserved;
    double center[3];       /* Surface.center (RT:1063) */
    double normal[3];       /* FlatSurface/PlaneMirror/PerfectLens .normal (RT:1320, 1389, 1576) */
    double input_axis[3];   /* Surface.input_axis (RT:1054): front-side test, sphere aperture axis */
    double radius;          /* SphericalSurface.radius (signed, RT:1445) */
    double radius_sq;       /* radius**2 exactly as the host evaluates it (RT:1499) */
    double aperture;        /* Surface.aperture_rad (RT:1069) */
    double focal_len;       /* PerfectLens.focal_len */
    double sin_alpha;       /* numpy.sin(PerfectLens.alpha) (RT:1758-1759) */
    double on_tol;          /* on-surface tolerance; 1e-12 reproduces RT:1343/1408/1528 */
} rtpb_surface;

typedef struct rtpb_material {
    int32_t kind;           /* RTPB_CONSTANT ... */
    int32_t table_len;      /* RTPB_TABLE: number of (wavelength, n) pairs */
    double c[6];            /* coefficients, see kinds */
    const double* table;    /* RTPB_TABLE: host pointer to table_len pairs {wavelength, n}, any order
                               (the library sorts them; lookups are binary searches); a NaN
                               wavelength key gives n(NaN).  Copied at plan creation. */
} rtpb_material;

typedef struct rtpb_plan rtpb_plan;   /* opaque: lowered system resident on the GPU(s) */

/* ---- library -------------------------------------------------------------------------------- */
int rtpb_abi_version(void);
const char* rtpb_last_error(void);
/* Number of visible GPUs (0 when none; never an error). */
int rtpb_device_count(void);
/* Release every device resource the library holds (plans must be destroyed first). */
int rtpb_shutdown(void);

/* ---- history buffers (ABI 5, stream-ordered since ABI 6) ---------------------------------------- */
/* Output buffers for large histories.  The 2S+1 planes of a history are written concurrently, and that
   write pattern runs 15-45 % slower into some physical placements -- physically contiguous memory in
   particular, which the first large allocations of a process on an unfragmented card often are -- while a
   plain fill of the same memory does not.  rtpb_buffer_alloc maps the buffer's physical
   memory in `chunk_bytes` chunks (0: 64 MiB) placed in the virtual range in a shuffled order (`seed`), so
   every buffer gets the fast rate.  The buffer is device memory like any other (pass `*ptr` to rtpb_trace).
   Streams -- PyTorch caching-allocator semantics, made explicit:
     * a buffer is allocated for `stream` (a hipStream_t, NULL = the device's null stream);
     * rtpb_buffer_record_stream(ptr, s) marks a use of the live buffer containing `ptr` on another stream
       `s` (returns 1, not an error, when `ptr` is not inside a live history buffer);
     * rtpb_buffer_free never blocks: it records an event on the allocation stream and on every recorded
       stream and keeps the buffer, still mapped, in a per-device pool;
     * the next rtpb_buffer_alloc of the same size on that device returns it and makes ITS stream wait for
       those events on the device (hipStreamWaitEvent): nothing the new owner queues can touch the memory
       before the previous owner's recorded uses have finished.
   The pool keeps the most recently freed buffer per device (rtpb_set_tuning("buffer_pool_buffers", k)
   keeps k, 0 none); an older one retires, still mapped.  Freeing and pooled allocations never block (ABI 8):
   retired buffers are unmapped and their physical memory released by the next allocation that maps new
   memory (after a device synchronisation; not while that allocation's stream is capturing a graph), by
   rtpb_buffer_trim and by rtpb_shutdown; their virtual ranges stay reserved, never reused.  rtpb_buffer_trim
   -- and rtpb_shutdown, and an allocation that finds the device full -- waits for the recorded uses and
   releases every pooled and retired buffer.  rtpb_buffer_held reports the bytes and buffers the pool still holds on `device`
   (-1: all devices).
   rtpb_buffer_dlpack wraps the whole buffer as a C-contiguous DLPack (v0.8 DLManagedTensor, device type
   ROCm) tensor of `ndim` extents `shape` and element type `dtype` (RTPB_F64 / RTPB_F32); ownership passes
   to the importer, whose call of the managed tensor's deleter frees the buffer.  rtpb_buffer_dlpack_discard
   runs that deleter for a managed tensor no importer consumed.  Replaces nothing in the reference (NumPy
   allocates its histories itself, RT:1229-1232). */
int rtpb_buffer_alloc(int32_t device, uint64_t bytes, uint64_t chunk_bytes, uint64_t seed, void* stream, void** ptr,
                      void** handle);
int rtpb_buffer_free(void* handle);
int rtpb_buffer_record_stream(const void* ptr, void* stream);
int rtpb_buffer_trim(void);
int rtpb_buffer_held(int32_t device, uint64_t* bytes, int32_t* buffers);
int rtpb_buffer_dlpack(void* handle, int32_t ndim, const int64_t* shape, int32_t dtype, void** managed);
int rtpb_buffer_dlpack_discard(void* managed);

/* ---- torch MemPool segments (ABI 7) ------------------------------------------------------------- */
/* The same shuffled-chunk memory as the segment allocator of PyTorch's caching allocator:
       torch.cuda.MemPool(torch.cuda.memory.CUDAPluggableAllocator("librtpb.so", "rtpb_torch_alloc",
                                                                    "rtpb_torch_free").allocator())
   (torch's alloc_fn / free_fn signatures: void* (size_t, int, hipStream_t), void (void*, size_t, int,
   hipStream_t)).  torch then caches, reuses stream-ordered (Tensor.record_stream), counts
   (torch.cuda.memory_allocated) and releases (empty_cache / out of memory) those segments itself; the library
   only maps a fresh buffer of `size` bytes (NULL on failure) and, on free, synchronises the device and unmaps
   it.  ray_trace_pb_amd's default device histories come from such a pool (_engine.history_pool).
   rtpb_buffer_stats fills up to n of: [0] live torch-pool segment bytes on `device` (-1: all), [1] their
   count, [2] reserved virtual bytes of released mappings (never reused), [3] their count,
   [4] buffers allocated with plain hipMalloc because [2] reached rtpb_set_tuning("buffer_dead_va_limit"),
   [5] torch segments allocated, [6] torch segments freed, [7] the dead-VA limit in bytes. */
void* rtpb_torch_alloc(int64_t size, int32_t device, void* stream);
void rtpb_torch_free(void* ptr, int64_t size, int32_t device, void* stream);
int rtpb_buffer_stats(int32_t device, uint64_t* out, int32_t n);

/* ---- plans: reference System + initial/final materials, lowered ----------------------------- */
/* Validates and stores the system.  `nmat` must equal `nsurf + 1` (RT:653-656: initial material,
   System.materials, final material).  `dtype` is the STORAGE type of the output history, RTPB_F64 or
   RTPB_F32; arithmetic is always float64 (the reference's numerics).  The input rays keep their own
   element type (`in_dtype` of the trace calls): float64 rays traced into an RTPB_F32 plan give the
   reference's float64 history rounded once to float32 (nothing is rounded before the arithmetic), and
   float32 rays are widened exactly, as NumPy promotes them in the reference. */
int rtpb_plan_create(const rtpb_surface* surfaces, int32_t nsurf,
                     const rtpb_material* materials, int32_t nmat,
                     int32_t dtype, rtpb_plan** plan_out);
int rtpb_plan_destroy(rtpb_plan* plan);

/* ---- tracing on device-resident buffers ----------------------------------------------------- */
/* Trace n_rays rays through the whole plan on `device`, asynchronously on `stream` (a hipStream_t,
   NULL = the device's null stream).
     rays_in          device pointer, n_rays rays in `in_layout` with elements of type `in_dtype`
                      (RTPB_F64 / RTPB_F32; SOA input must use the plan's dtype); SOA fields are
                      `in_field_stride` elements apart (>= n_rays).
     out              device pointer to slot 0 of the output; slots are `out_plane_stride` elements
                      apart (>= 8*n_rays); SOA fields are `out_field_stride` elements apart.
     plane_mask_lo/hi bits 0..63 / 64..127 select history planes 0..2S (see above).
   The output's element type is the plan's dtype. */
int rtpb_trace(const rtpb_plan* plan, int32_t device,
               const void* rays_in, int32_t in_dtype, int64_t n_rays, int32_t in_layout, int64_t in_field_stride,
               void* out, int32_t out_layout, int64_t out_plane_stride, int64_t out_field_stride,
               uint64_t plane_mask_lo, uint64_t plane_mask_hi, void* stream);
/* rtpb_trace plus a table-miss flag: `table_miss` (device pointer to one int32, may be NULL) is set to
   1 by the launch when some ray's wavelength is not a key of some RTPB_TABLE material of the plan (that
   ray's n would be NaN, unlike the material's own n()).  The caller zeroes it before the call and reads
   it after the stream has completed.  Lets a caller trace optimistically with the table keys of a
   previous bundle and re-trace with the bundle's own keys only on a miss (bit-identical either way). */
int rtpb_trace_checked(const rtpb_plan* plan, int32_t device,
                       const void* rays_in, int32_t in_dtype, int64_t n_rays, int32_t in_layout,
                       int64_t in_field_stride, void* out, int32_t out_layout, int64_t out_plane_stride,
                       int64_t out_field_stride, uint64_t plane_mask_lo, uint64_t plane_mask_hi, void* stream,
                       int32_t* table_miss);

/* rtpb_trace_checked with its arguments in one struct (same fields, same meaning; table_miss may be NULL).  For
   bindings whose per-argument marshalling costs more than the call (ctypes: ~0.2 us per argument): the caller keeps
   a filled struct per (plan, shape, planes, stream) and updates the buffer pointers between calls. */
typedef struct rtpb_trace_call {
    const rtpb_plan* plan;
    const void* rays_in;
    void* out;
    void* stream;
    int32_t* table_miss;
    int64_t n_rays;
    int64_t in_field_stride;
    int64_t out_plane_stride;
    int64_t out_field_stride;
    uint64_t plane_mask_lo;
    uint64_t plane_mask_hi;
    int32_t device;
    int32_t in_dtype;
    int32_t in_layout;
    int32_t out_layout;
} rtpb_trace_call;
int rtpb_trace_packed(const rtpb_trace_call* call);

/* ---- one-shot calls (the replacement of RT:658-659 without a plan handle) ------- */
/* The whole system in one call: `surfaces` (nsurf) and `materials` (nmat = nsurf + 1: initial material,
   System.materials, final material -- RT:653-656) as for rtpb_plan_create, device buffers as for rtpb_trace.
     rays_in  device pointer, n_rays x 8 AOS records of double (rtpb_trace_f64) / float (rtpb_trace_f32)
     out      device pointer: the history in the same element type (float: the float64 trace rounded once
              on store, float rays widened exactly -- as rtpb_trace with an RTPB_F32 plan)
     plane_mask_flags  0 = every plane 0..2S, (2S+1) x n_rays x 8 AOS: the reference's return value
              (RT:1229-1232); RTPB_PLANES_FINAL = plane 2S alone (n_rays x 8); RTPB_OUT_SOA = planes stored
              [8][n_rays] instead of [n_rays][8].  Other bits: RTPB_E_INVALID.  (Any other plane
              selection: rtpb_plan_create + rtpb_trace.)
   Asynchronous on `hip_stream` (NULL = the device's null stream).  The system is lowered into a plan once
   and cached by content (every descriptor byte and the (wavelength, n) pairs of RTPB_TABLE materials; the
   16 most recently used systems), so repeated calls with one system cost a compare of its descriptors.
   rtpb_oneshot_plans returns the number of cached plans; rtpb_oneshot_clear drops them (a plan still in
   use by a call on another thread is destroyed when that call returns; rtpb_shutdown clears them too). */
#define RTPB_PLANES_FINAL 0x1u
#define RTPB_OUT_SOA 0x2u
int rtpb_trace_f64(const rtpb_surface* surfaces, int32_t nsurf, const rtpb_material* materials, int32_t nmat,
                   const double* rays_in, int64_t n_rays, double* out, uint32_t plane_mask_flags, int32_t device,
                   void* hip_stream);
int rtpb_trace_f32(const rtpb_surface* surfaces, int32_t nsurf, const rtpb_material* materials, int32_t nmat,
                   const float* rays_in, int64_t n_rays, float* out, uint32_t plane_mask_flags, int32_t device,
                   void* hip_stream);
int rtpb_oneshot_plans(void);
void rtpb_oneshot_clear(void);

/* ---- tracing host buffers (NumPy in, NumPy out), sharded over several GPUs ------------------ */
/* rays_in: host, n_rays x 8 AOS of `in_dtype`.  out: host, nslots x n_rays x 8 AOS of the plan's dtype
   (nslots = popcount of the mask).
   Rays are split into contiguous index ranges, one per listed device (NULL/0 devices = device 0),
   each traced by its own host thread with chunked, double-buffered H2D / kernel / D2H copies.
   Synchronous: returns when `out` is complete. */
int rtpb_trace_host(const rtpb_plan* plan, const void* rays_in, int32_t in_dtype, int64_t n_rays, void* out,
                    uint64_t plane_mask_lo, uint64_t plane_mask_hi,
                    const int32_t* devices, int32_t n_devices);

/* ---- device ray generators (reference RT:45-161), written straight into device memory -------- */
/* get_ray_fan(pt, theta_max, n_thetas, wavelength, nphis, center_ray): ray k = iphi*n_thetas+itheta.
   These two evaluate cos/sin with the device libm (within 1 ulp of the host's); the *_tables variants
   below are bit-exact against the caller's NumPy. */
int rtpb_ray_fan(int32_t device, int32_t dtype, void* rays_out, const double pt[3], double theta_max,
                 int64_t n_thetas, int64_t nphis, const double center_ray[3], double wavelength,
                 void* stream);

/* get_collimated_rays(pt, displacement_max, n_disps, wavelength, nphis, phi_start, normal) (RT:99-161):
   ray k = idisp*nphis + iphi; `normal` must be a unit vector. */
int rtpb_collimated_rays(int32_t device, int32_t dtype, void* rays_out, const double pt[3], double displacement_max,
                         int64_t n_disps, int64_t nphis, double phi_start, const double normal[3], double wavelength,
                         void* stream);

/* Same two generators with every host-side constant supplied by the caller, so the device output is
   bit-identical to the caller's own NumPy evaluation of RT:45-161: ex/ey (or n1/n2) basis vectors,
   (cos, sin) pairs of the linspace thetas (2*n_thetas doubles) and of the phis (2*nphis doubles), and
   the offsets (n_disps doubles).  Tables are HOST pointers, copied before the call returns. */
int rtpb_ray_fan_tables(int32_t device, int32_t dtype, void* rays_out, const double pt[3], int64_t n_thetas,
                        int64_t nphis, const double center_ray[3], const double ex[3], const double ey[3],
                        const double* theta_cos_sin, const double* phi_cos_sin, double wavelength, void* stream);
int rtpb_collimated_rays_tables(int32_t device, int32_t dtype, void* rays_out, const double pt[3], int64_t n_disps,
                                int64_t nphis, const double normal[3], const double n1[3], const double n2[3],
                                const double* offsets, const double* phi_cos_sin, double wavelength, void* stream);
/* ABI 7: the same with one wavelength per ray -- the reference's "either floating point or an array the same
   size as n_disps * nphis" (RT:115; rays[:, 7] = wavelengths, RT:94 / RT:159).  `wavelengths` is a DEVICE
   pointer to n_thetas*nphis (n_disps*nphis) float64 values in ray-index order, 8-byte aligned, read by the
   kernel (stream-ordered); everything else as above. */
int rtpb_ray_fan_tables_wl(int32_t device, int32_t dtype, void* rays_out, const double pt[3], int64_t n_thetas,
                           int64_t nphis, const double center_ray[3], const double ex[3], const double ey[3],
                           const double* theta_cos_sin, const double* phi_cos_sin, const double* wavelengths,
                           void* stream);
int rtpb_collimated_rays_tables_wl(int32_t device, int32_t dtype, void* rays_out, const double pt[3],
                                   int64_t n_disps, int64_t nphis, const double normal[3], const double n1[3],
                                   const double n2[3], const double* offsets, const double* phi_cos_sin,
                                   const double* wavelengths, void* stream);

/* propagate_ray2plane(rays, normal, center, material, exclude_backward_propagation) (RT:241-306) on
   device rays (AOS n x 8).  normal / center: DEVICE pointers to 3 doubles (broadcast) or n x 3 doubles
   (*_per_ray = 1).  ts_out (device, n doubles) may be NULL.  workspace: device bytes for the material
   descriptor (>= 256 + 16 * max(table_len, 1)); the call synchronises `stream` after staging it. */
int rtpb_propagate_plane(int32_t device, int32_t dtype, const void* rays_in, int64_t n_rays, const double* normal,
                         int32_t normal_per_ray, const double* center, int32_t center_per_ray,
                         const rtpb_material* material, int32_t exclude_backward, void* rays_out, double* ts_out,
                         void* workspace, int64_t workspace_bytes, void* stream);

/* ---- user Surface subclasses with their own geometry (reference plugin point RT:1071-1156) ----- */
/* A Surface subclass that keeps RefractingSurface.propagate (RT:1160-1234) or
   ReflectingSurface.propagate (RT:1238-1303) but supplies its own get_intersect / get_normal /
   is_pt_on_surface.  The caller evaluates those three hooks; the library does the rest of propagate
   on the device.  `plan` holds ONE surface (only its input_axis is read) and TWO materials (the
   media before / after the surface); buffers are device pointers in the plan's storage type, rays
   AOS n x 8, normals n x 3.
   rtpb_front_side: hits_out = hits with every row NaN where rays.d . input_axis < 0 (RT:1184-1192);
     hits_out may equal hits.
   rtpb_interact: out = Snell refraction (mode RTPB_REFRACT, n1/n2 from the plan's materials at the
     hit's wavelength, RT:1194-1221) or reflection (RTPB_REFLECT, RT:1266-1289) of `hits` about
     `normals`, with position NaN where the direction is NaN (TIR) and the whole row NaN where
     on_surface[i] == 0 (RT:1225-1226; on_surface NULL = all on). */
int rtpb_front_side(const rtpb_plan* plan, int32_t device, const void* rays, const void* hits, int64_t n,
                    void* hits_out, void* stream);
int rtpb_interact(const rtpb_plan* plan, int32_t device, int32_t mode, const void* hits, const void* normals,
                  const uint8_t* on_surface, int64_t n, void* out, void* stream);

/* ---- device analysis ------------------------------------------------------------------------- */
/* intersect_rays(ray1, ray2) (RT:164-238) on device rays (AOS, n x 8; a length-1 side broadcasts).
   pts_out: max(n1, n2) x 3 intersection points, NaN where the rays do not meet within 1e-12. */
int rtpb_intersect_rays(int32_t device, int32_t dtype, const void* ray1, int64_t n1, const void* ray2, int64_t n2,
                        void* pts_out, void* stream);
/* Spot statistics of one (N, 8) AOS plane split into n_groups contiguous groups of group_size rays
   (e.g. one group per (field point, wavelength) fan).  Rays with non-finite x or y are skipped.
   stats_out (device, n_groups x 7 doubles): count, sum x, sum y, sum z, sum x^2, sum y^2, sum x*y.
   Deterministic (fixed-order two-pass reduction).  workspace: device doubles,
   >= n_groups * ceil(group_size / 256) * 7. */
int rtpb_spot_stats(int32_t device, int32_t dtype, const void* plane, int64_t group_size, int64_t n_groups,
                    double* workspace, int64_t workspace_len, double* stats_out, void* stream);

/* Fused spot-diagram sweep (the C5 workload): for every group g the fan
   get_ray_fan(pt_g, theta_max, n_thetas, wavelength_g, nphis, center_ray) (RT:45-96) is generated,
   traced through `plan` (final state only) and reduced to the 7 statistics of rtpb_spot_stats -- one
   kernel, nothing but the statistics reaches HBM.  group_params: HOST, n_groups x {x, y, z, wavelength};
   ex/ey and the (cos, sin) tables as for rtpb_ray_fan_tables (host).  workspace: device doubles,
   >= n_groups * ceil(n_thetas*nphis / 256) * 7.  stats_out: device, n_groups x 7.  The statistics are
   bit-identical to rtpb_ray_fan_tables + rtpb_trace (final plane) + rtpb_spot_stats in the plan's
   storage type.  Groups with the same field point (bit for bit) are swept together -- each ray generated once
   and, when the first surface is a refracting flat or sphere, its wavelength-independent part computed once --
   so a call should hold all the wavelengths of its field points (order does not matter). */
int rtpb_spot_sweep(const rtpb_plan* plan, int32_t device, int64_t n_groups, const double* group_params,
                    int64_t n_thetas, int64_t nphis, const double center_ray[3], const double ex[3],
                    const double ey[3], const double* theta_cos_sin, const double* phi_cos_sin, double* workspace,
                    int64_t workspace_len, double* stats_out, void* stream);

/* ---- pupil-phase interpolation (scripts/2022_02_06_perfect_imaging_system_psf.py:90-105) */
/* A 2-D Delaunay triangulation with one value per vertex, in scipy.spatial.Delaunay's representation,
   plus a uniform cell index (CSR lists of the triangles whose bounding box meets each cell, in
   increasing triangle order).  All pointers are device pointers. */
typedef struct rtpb_triangulation {
    int64_t n_tri;
    const double* transform;    /* n_tri x 3 x 2: Delaunay.transform (2x2 inverse, then the offset row) */
    const int32_t* simplices;   /* n_tri x 3 vertex indices */
    const double* values;       /* value of each vertex */
    int32_t cells_x, cells_y;   /* cell (cx, cy) covers [x0 + cx*cell_w, +cell_w) x [y0 + cy*cell_h, +cell_h) */
    double x0, y0, cell_w, cell_h;
    const int32_t* cell_start;  /* cells_x*cells_y + 1 offsets into cell_tris; cell id = cy*cells_x + cx */
    const int32_t* cell_tris;
} rtpb_triangulation;

/* griddata(points, values, (xx, yy), method='linear') on the grid meshgrid(xs, ys) (point (iy, ix) =
   (xs[ix], ys[iy]), row-major), with scipy's LinearNDInterpolator arithmetic: the first triangle whose
   barycentric coordinates lie in [-eps, 1+eps] (eps = 100 DBL_EPSILON), c0/c1 from the transform and
   c2 = (1 - c0) - c1, value = ((0 + c0 v0) + c1 v1) + c2 v2; NaN outside the hull.  Optionally fused
   with the pupil field of the script: field = exp(i phase), 0 where phase is NaN or
   sqrt(x^2 + y^2) > radius.  phase_out (ny*nx doubles) and/or field_out (ny*nx interleaved complex
   doubles) may be NULL.  xs, ys: device arrays. */
int rtpb_grid_interpolate(int32_t device, const rtpb_triangulation* tri, const double* xs, int64_t nx,
                          const double* ys, int64_t ny, double radius, double* phase_out, double* field_out,
                          void* stream);

/* ---- distinct wavelengths of a device-resident bundle (keys of the plan's RTPB_TABLE materials) -- */
/* Replaces the host-side np.unique of the wavelength column that tabulated materials need
   (MAT:128-144 Ebaf11 and user Material.n are evaluated by the host at exactly these wavelengths).
   col: device pointer to the first wavelength, `stride` elements between consecutive rays (8 for an
   (N, 8) AoS bundle), n values of `dtype` (RTPB_F64 / RTPB_F32, widened exactly).  table: device buffer
   of `table_slots` uint64 (a power of two); max_keys <= table_slots / 2; count: one device uint32.
   Asynchronous on `stream`.  Afterwards the table holds the distinct keys as float64 bit patterns (all
   NaNs as one quiet-NaN key, -0.0 as +0.0) in arbitrary order, empty slots = all-ones; *count is the
   number of keys, or > max_keys when there are more (the caller then sorts instead). */
int rtpb_distinct_keys(int32_t device, const void* col, int32_t dtype, int64_t n, int64_t stride, uint64_t* table,
                       int32_t table_slots, int32_t max_keys, uint32_t* count, void* stream);

/* ---- tuning knobs (benchmarks / A-B tests; process-wide) ------------------------------------ */
/* "aos_staging": 1 (default) = AOS planes are written through a per-wave LDS tile so every global
   store instruction writes 1 KiB contiguous; 0 = direct 16-byte stores at the record stride.
   "nt_stores": 1 (default) = non-temporal global stores for the staged AOS tiles (the history is
   streamed out and never re-read by the kernel); 0 = default cache policy.
   "stage_input": 1 = also load AOS input records through the LDS tile (1 KiB per load instruction);
   0 (default) = 4 x 16-byte loads per lane.
   "host_chunk_mib": input + output bytes per pipelined chunk of rtpb_trace_host (default 128).
   "indexed_materials": 1 (default) = plans created from now on whose TABLE materials all share one
   key set (and that have no POLY6 material) also tabulate every other material at those keys, so the
   kernel reads n from LDS instead of evaluating Sellmeier dispersion per surface (bit-identical: the
   host evaluates the kernel's own material_n); 0 = evaluate per surface.
   "buffer_pool_buffers": freed history buffers kept mapped per device for reuse (default 1, 0..1024).
   "buffer_dead_va_limit": reserved virtual bytes of released buffer mappings (never reused) beyond which new
                           history buffers are plain hipMalloc allocations (default 32 TiB). */
int rtpb_set_tuning(const char* key, int64_t value);

/* ---- kernel timing (benchmarks) ------------------------------------------------------------- */
/* While enabled on the calling thread, every trace kernel this thread launches is bracketed by a pair
   of HIP events recorded on the kernel's own stream.  rtpb_timing_collect() waits for them and
   returns the summed kernel time (ms) and launch count since the last collect, then resets. */
int rtpb_timing_enable(int32_t on);
int rtpb_timing_collect(double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* RTPB_H */
