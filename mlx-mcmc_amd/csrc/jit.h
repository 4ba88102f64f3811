// jit.h — the expression-term JIT (jit.hip): per-program compiled EX
// instantiations of the tape kernels.
#pragma once
#include <string>

#include "host.h"

// MC_EXPR_JIT / mc_debug_expr_jit
bool jit_enabled();
// Launch `kernel` (a name expression, e.g. "mc::k_hmc<8, true, true>")
// compiled with the program's expression terms; *used = false (and MC_OK)
// when the JIT is off, the program has no expression terms, or its
// compilation failed: the caller then launches the interpreter's kernel.
int jit_launch(const mc_program* p, const std::string& kernel, unsigned grid, unsigned block,
               size_t lds, hipStream_t st, void** args, bool* used);
// The compiled `kernel` of the program (loaded on the current device);
// *fn = nullptr (and MC_OK) when the JIT is off, the program has no
// expression terms, or the compilation failed.
int jit_function(const mc_program* p, const std::string& kernel, hipFunction_t* fn);
// The last compilation failure of the program ("" if none).
std::string jit_error(const mc_program* p);
void jit_free(mc_program* p);
