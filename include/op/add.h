// add.h — the reference include/op/add.h name; all operators are declared in ops.h.
#pragma once
#include "ops.h"
