// tiresias_amd — one production gemm8p variant per translation unit (gemm8p.h):
// the 128x128 tile with its K range split over two wave groups of one block.
#include "tam/gemm8p.h"

namespace tam {
TAM_P8_KS2_INST(128, 128, 2, true, true)
}  // namespace tam
