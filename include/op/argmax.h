// argmax.h — the reference include/op/argmax.h name; all operators are declared in ops.h.
#pragma once
#include "ops.h"
