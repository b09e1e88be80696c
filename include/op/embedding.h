// embedding.h — the reference include/op/embedding.h name; all operators are declared in ops.h.
#pragma once
#include "ops.h"
