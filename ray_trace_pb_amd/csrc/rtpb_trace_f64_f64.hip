// Trace kernel variants for f64 input rays and f64 history storage (see rtpb_trace_kernel.h).
#include "rtpb_trace_kernel.h"

namespace rtpbi {
template hipError_t launch_trace<double, double>(const TraceArgs<double, double>&, int, int, int, hipStream_t);
}  // namespace rtpbi
