/* placeholder: OSQP-default ADMM restatement (CPU baseline) */
#include "f110_oracle.h"
