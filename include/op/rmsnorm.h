// rmsnorm.h — the reference include/op/rmsnorm.h name; all operators are declared in ops.h.
#pragma once
#include "ops.h"
