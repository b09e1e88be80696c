// mha.h — the reference include/op/mha.h name; all operators are declared in ops.h.
#pragma once
#include "ops.h"
