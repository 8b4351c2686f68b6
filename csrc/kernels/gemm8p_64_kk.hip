// tiresias_amd — one production gemm8p variant per translation unit (gemm8p.h).
#include "tam/gemm8p.h"

namespace tam {
TAM_P8_INST(64, 128, 2, true, true)
}  // namespace tam
