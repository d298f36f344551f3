// bg_debug.h — the library's explicit debug options (bgx_debug_option, include/bgx.h).
// The product path never reads the environment: the exact alternative paths the GPU
// tests compare (the 2-ply enumerator / evaluator / pool variants, the policy kernel's
// tile-skip forms, the dispatch order) and the diagnostics are selected only through
// bgx_debug_option.  Options read at engine creation keep the engine's value.
#pragma once
#include <string>

// The value set for `name` by bgx_debug_option, or "" when unset.
std::string bgx_dbg(const char* name);
// bgx_dbg(name) as an integer, or `dflt` when unset.
long long bgx_dbg_int(const char* name, long long dflt);
