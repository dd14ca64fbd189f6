// Launch-timing hooks (see drt_profile_enable in include/drt.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace drt {

enum ProfFamily { PROF_SCAN = 0, PROF_SAMPLE = 1, PROF_SELECT = 2, PROF_MERGE = 3, PROF_GEMM = 4, PROF_N = 5 };

// Returns a pair of events to record around one launch, or {nullptr,nullptr}
// when the family is not being profiled.
struct ProfPair {
  hipEvent_t a, b;
};
ProfPair prof_begin(int family, hipStream_t s);
void prof_end(const ProfPair& p, hipStream_t s);

}  // namespace drt
