// dwpw_mfma_k5s2.hip -- the 5x5 stride-2 instances of the MFMA dwpw forms (dwpw_mfma.h).
#include "dwpw_mfma.h"

namespace zr {

const char *dwpw_layout_k5s2(const DwPwParams &p, const DwPwLayout &l, hipStream_t s) { return dwpw_layout<5, 2>(p, l, s); }

}  // namespace zr
