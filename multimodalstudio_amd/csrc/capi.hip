// Library-level C-ABI entry points: version string and last-error text.
#include "common.h"

MMS_EXPORT const char* mms_version() { return "mms_hip 0.1 (gfx950)"; }

MMS_EXPORT const char* mms_last_error() { return mms::err_buf(); }
