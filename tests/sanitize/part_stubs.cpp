// Stand-ins for the per-window-side parts of libgw_engine.so (gw_engine.hip,
// -DGW_PART_S): the sanitizer build of the host part (tests/test_sanitizers.py)
// links these instead of the kernels, so that gw_create's validation and table
// building run under AddressSanitizer / UBSan without device code.  Every
// launch or attribute call reports an error.
#include <hip/hip_runtime.h>

#define GW_STUB_PART(S)                                                                       \
    hipError_t gw_part_launch_##S(int, unsigned, unsigned, size_t, hipStream_t, const void*,  \
                                  hipEvent_t, hipEvent_t) { return hipErrorInvalidValue; }    \
    hipError_t gw_part_attr_##S(int, size_t) { return hipErrorInvalidValue; }                 \
    hipError_t gw_part_occ_##S(int, unsigned, size_t, int*) { return hipErrorInvalidValue; }
GW_STUB_PART(1) GW_STUB_PART(3) GW_STUB_PART(5) GW_STUB_PART(7)
GW_STUB_PART(9) GW_STUB_PART(11) GW_STUB_PART(13) GW_STUB_PART(15)
GW_STUB_PART(0)
