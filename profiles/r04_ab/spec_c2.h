// A/B build (profiles/build_variant.sh, force-included): the analyze body specialised for bench.py's
// c2 configuration, as a JIT kernel would be (lt_jit.h LT_SPEC_*): 30 years, no cloud mask, labels
// only, one GD rule without filters, line_cost 10. Timing builds only: any other configuration
// launched on it would be analysed wrongly.
#pragma once
#include "../../include/lt_abi.h"
#define LT_SPEC_Y 30
#define LT_SPEC_MASKED 0
#define LT_SPEC_YEAR_OUT 0
#define LT_SPEC_NRULES 1
#define LT_SPEC_PRE_MODE 0
#define LT_SPEC_LINE_COST 10.0
__device__ constexpr lt_rule lt_spec_rules[1] = {{LT_CT_GD, LT_Q_UNSET, LT_Q_UNSET, LT_Q_UNSET,
                                                   0.0, 0.0, 0.0, 1, 0}};
