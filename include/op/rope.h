// rope.h — the reference include/op/rope.h name; all operators are declared in ops.h.
#pragma once
#include "ops.h"
