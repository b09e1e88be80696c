// swiglu.h — the reference include/op/swiglu.h name; all operators are declared in ops.h.
#pragma once
#include "ops.h"
