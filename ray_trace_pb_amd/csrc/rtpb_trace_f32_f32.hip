// Trace kernel variants for f32 input rays and f32 history storage, plan-feature group 0 (feat 0, 1, 4, 5, 33) (see rtpb_trace_kernel.h).
#include "rtpb_trace_kernel.h"

namespace rtpbi {
template hipError_t launch_trace_group<float, float, 0>(const TraceArgs<float, float>&, int, int, int, hipStream_t);
}  // namespace rtpbi
