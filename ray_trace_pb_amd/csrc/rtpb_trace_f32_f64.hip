// Trace kernel variants for f32 input rays and f64 history storage (see rtpb_trace_kernel.h).
#include "rtpb_trace_kernel.h"

namespace rtpbi {
template hipError_t launch_trace<float, double>(const TraceArgs<float, double>&, int, int, int, hipStream_t);
}  // namespace rtpbi
