// rtpb_oneshot.hip -- the one-shot entry points of SURVEY.md §8(b) (ABI 8): rtpb_trace_f64 / rtpb_trace_f32 take
// the system descriptors and the device buffers in ONE call, the literal replacement of System.ray_trace's surface
// loop (RT:658-659) for a caller that does not want to manage plans.
//
// They are thin wrappers over the plan API: the (surfaces, materials, storage type) of a call are lowered into a
// plan once and cached by CONTENT -- the bytes of every descriptor plus the (wavelength, n) pairs of TABLE
// materials -- so repeated calls with the same system pay a compare of a few hundred bytes, not the
// lowering (the exact on-surface thresholds are bisections, ~10 us per surface) or the descriptor upload.  The cache
// keeps the kOneShotPlans most recently used plans; a plan evicted while another thread still traces with it is
// destroyed by its last user (shared ownership).
#include "rtpb_internal.h"

#include <list>
#include <memory>

using namespace rtpbi;

namespace {

constexpr size_t kOneShotPlans = 16;

struct PlanDeleter {
    void operator()(rtpb_plan* p) const { (void)rtpb_plan_destroy(p); }
};
using PlanRef = std::shared_ptr<rtpb_plan>;

std::mutex g_oneshot_mu;
std::list<std::pair<std::string, PlanRef>> g_oneshot;      // most recently used first

// The content key of a call: storage type, the descriptors (table pointers replaced by their pairs).
std::string content_key(const rtpb_surface* s, int32_t nsurf, const rtpb_material* m, int32_t nmat, int32_t dtype) {
    std::string k;
    k.reserve(8 + sizeof(rtpb_surface) * static_cast<size_t>(nsurf) + sizeof(rtpb_material) * static_cast<size_t>(nmat));
    k.append(reinterpret_cast<const char*>(&dtype), sizeof dtype);
    k.append(reinterpret_cast<const char*>(&nsurf), sizeof nsurf);
    k.append(reinterpret_cast<const char*>(s), sizeof(rtpb_surface) * static_cast<size_t>(nsurf));
    for (int32_t i = 0; i < nmat; ++i) {
        rtpb_material c = m[i];
        c.table = nullptr;
        k.append(reinterpret_cast<const char*>(&c), sizeof c);
        if (m[i].kind == RTPB_TABLE && m[i].table && m[i].table_len > 0)
            k.append(reinterpret_cast<const char*>(m[i].table), sizeof(double) * 2 * static_cast<size_t>(m[i].table_len));
    }
    return k;
}

// The cached plan of this content (created on a miss); rc != RTPB_OK with the message set on failure.
int cached_plan(const rtpb_surface* s, int32_t nsurf, const rtpb_material* m, int32_t nmat, int32_t dtype, PlanRef* out) {
    if (nsurf < 0 || (nsurf > 0 && !s)) return fail(RTPB_E_INVALID, "bad surfaces array");
    if (nsurf > RTPB_MAX_SURFACES)
        return fail(RTPB_E_LIMIT, "more than RTPB_MAX_SURFACES (" + std::to_string(RTPB_MAX_SURFACES) + ") surfaces");
    if (nmat != nsurf + 1 || !m) return fail(RTPB_E_INVALID, "length of materials should be len(surfaces) + 1");
    std::string key = content_key(s, nsurf, m, nmat, dtype);
    {
        std::lock_guard<std::mutex> lk(g_oneshot_mu);
        for (auto it = g_oneshot.begin(); it != g_oneshot.end(); ++it) {
            if (it->first == key) {
                g_oneshot.splice(g_oneshot.begin(), g_oneshot, it);
                *out = it->second;
                return RTPB_OK;
            }
        }
    }
    rtpb_plan* p = nullptr;
    const int rc = rtpb_plan_create(s, nsurf, m, nmat, dtype, &p);
    if (rc != RTPB_OK) return rc;
    PlanRef ref(p, PlanDeleter{});
    std::lock_guard<std::mutex> lk(g_oneshot_mu);
    g_oneshot.emplace_front(std::move(key), ref);
    while (g_oneshot.size() > kOneShotPlans) g_oneshot.pop_back();     // destroyed by its last user
    *out = ref;
    return RTPB_OK;
}

int oneshot(const rtpb_surface* s, int32_t nsurf, const rtpb_material* m, int32_t nmat, int32_t dtype,
            const void* rays_in, int64_t n, void* out, uint32_t flags, int32_t device, void* stream) {
    if (flags & ~(RTPB_PLANES_FINAL | RTPB_OUT_SOA))
        return fail(RTPB_E_INVALID, "plane_mask_flags: unknown bits (RTPB_PLANES_FINAL | RTPB_OUT_SOA)");
    if (n < 0) return fail(RTPB_E_INVALID, "n_rays < 0");
    PlanRef plan;
    int rc = cached_plan(s, nsurf, m, nmat, dtype, &plan);
    if (rc != RTPB_OK) return rc;
    // planes: the whole history 0..2S (the reference's return value) or the final plane 2S alone
    const int last = 2 * nsurf;
    uint64_t lo = 0, hi = 0;
    if (flags & RTPB_PLANES_FINAL) {
        if (last < 64) lo = 1ull << last;
        else hi = 1ull << (last - 64);
    } else {
        lo = last >= 63 ? ~0ull : ((1ull << (last + 1)) - 1);
        hi = last >= 64 ? ((1ull << (last - 63)) - 1) : 0;
    }
    const int32_t ol = (flags & RTPB_OUT_SOA) ? RTPB_SOA : RTPB_AOS;
    // AOS planes of 8 n elements; SOA planes [8][n]: fields n apart
    return rtpb_trace(plan.get(), device, rays_in, dtype, n, RTPB_AOS, 0, out, ol, 8 * n, n, lo, hi, stream);
}

}  // namespace

extern "C" {

int rtpb_trace_f64(const rtpb_surface* surfaces, int32_t nsurf, const rtpb_material* materials, int32_t nmat,
                   const double* rays_in, int64_t n_rays, double* out, uint32_t plane_mask_flags, int32_t device,
                   void* hip_stream) {
    return oneshot(surfaces, nsurf, materials, nmat, RTPB_F64, rays_in, n_rays, out, plane_mask_flags, device,
                   hip_stream);
}

int rtpb_trace_f32(const rtpb_surface* surfaces, int32_t nsurf, const rtpb_material* materials, int32_t nmat,
                   const float* rays_in, int64_t n_rays, float* out, uint32_t plane_mask_flags, int32_t device,
                   void* hip_stream) {
    return oneshot(surfaces, nsurf, materials, nmat, RTPB_F32, rays_in, n_rays, out, plane_mask_flags, device,
                   hip_stream);
}

int rtpb_oneshot_plans(void) {
    std::lock_guard<std::mutex> lk(g_oneshot_mu);
    return static_cast<int>(g_oneshot.size());
}

void rtpb_oneshot_clear(void) {
    std::list<std::pair<std::string, PlanRef>> drop;
    {
        std::lock_guard<std::mutex> lk(g_oneshot_mu);
        drop.swap(g_oneshot);
    }
}

}  // extern "C"
