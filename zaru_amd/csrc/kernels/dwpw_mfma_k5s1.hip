// dwpw_mfma_k5s1.hip -- the 5x5 stride-1 instances of the MFMA dwpw forms (dwpw_mfma.h).
#include "dwpw_mfma.h"

namespace zr {

const char *dwpw_layout_k5s1(const DwPwParams &p, const DwPwLayout &l, hipStream_t s) { return dwpw_layout<5, 1>(p, l, s); }

}  // namespace zr
