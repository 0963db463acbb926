// Internal helpers shared by the C-ABI translation units.
#pragma once

// Records `msg` as rt_last_error() for this thread and returns `code`.
int rt_internal_set_error(int code, const char* msg);
