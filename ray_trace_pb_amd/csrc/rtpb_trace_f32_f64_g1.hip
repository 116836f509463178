// Trace kernel variants for f32 input rays and f64 history storage, plan-feature group 1 (feat 15, 16, 17) (see rtpb_trace_kernel.h).
#include "rtpb_trace_kernel.h"

namespace rtpbi {
template hipError_t launch_trace_group<float, double, 1>(const TraceArgs<float, double>&, int, int, int, hipStream_t);
}  // namespace rtpbi
