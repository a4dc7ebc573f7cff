// lgx_knobs.h — run-time dev knobs (A/B experiments) are compiled out of the product libraries.
// A product build ignores the environment: LGX_DEV_KNOB(name) is nullptr, so a stray variable
// cannot change the measured kernel. A dev build (-DLGX_DEV_KNOBS, build_native.build_variant)
// reads them.
#pragma once
#include <stdlib.h>

#ifdef LGX_DEV_KNOBS
#define LGX_DEV_KNOB(name) getenv(name)
#else
#define LGX_DEV_KNOB(name) ((const char*)nullptr)
#endif
