// matmul.h — the reference include/op/matmul.h name; all operators are declared in ops.h.
#pragma once
#include "ops.h"
