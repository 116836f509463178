// Trace kernel variants for f64 input rays and f64 history storage, plan-feature group 0 (feat 0, 1, 4, 5, 33) (see rtpb_trace_kernel.h).
#include "rtpb_trace_kernel.h"

namespace rtpbi {
template hipError_t launch_trace_group<double, double, 0>(const TraceArgs<double, double>&, int, int, int, hipStream_t);
}  // namespace rtpbi
