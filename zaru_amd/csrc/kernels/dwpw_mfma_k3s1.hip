// dwpw_mfma_k3s1.hip -- the 3x3 stride-1 instances of the MFMA dwpw forms (dwpw_mfma.h).
#include "dwpw_mfma.h"

namespace zr {

const char *dwpw_layout_k3s1(const DwPwParams &p, const DwPwLayout &l, hipStream_t s) { return dwpw_layout<3, 1>(p, l, s); }

}  // namespace zr
