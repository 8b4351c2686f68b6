// tiresias_amd — the A/B schedules of gemm8p (tools/ab_gemm8p_sched.py, tests).
#include "tam/gemm8p.h"

namespace tam {
TAM_P8_VARIANTS(TAM_P8_INST, 0)
TAM_P8_VARIANTS(TAM_P8_INST, 1)
TAM_P8_VARIANTS(TAM_P8_INST, 2)
TAM_P8_VARIANTS(TAM_P8_INST, 3)
TAM_P8_VARIANTS(TAM_P8_INST, 5)
}  // namespace tam
