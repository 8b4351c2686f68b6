// tiresias_amd — one production gemm8p variant per translation unit (gemm8p.h).
#include "tam/gemm8p.h"

namespace tam {
TAM_P8_INST(256, 256, 4, true, true)
}  // namespace tam
