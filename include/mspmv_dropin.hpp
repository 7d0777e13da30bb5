// mspmv_dropin.hpp -- drop-in replacement of the reference's CPU solvers by libmspmv.
//
// A reference driver (cpu_multicg.cpp, cpu_singlecg.cpp, verification/*) adds ONE line after
// its sparse_matrix.h / utils.h / work_2025/hyper_parameters.hpp includes:
//     #include "mspmv_dropin.hpp"
// compiles with -I<mspmv>/include -I<reference root> and links -lmspmv.  Its calls to
// CGSolveSingle / TestCGSolveSingle / CGSolveMultiple / TestCGMultipleRHS / OmpMergeCsrmm /
// IncompleteCholesky / TransposeCsr / PCGSolveMultiple / TestPCGMultipleRHS /
// SparseApproximateInversion / SPAISolveMultiple / TestCGMultipleSPAI then run on the MI355X, and
// its #include lines of work_2025/main/*.hpp (and the cg/spmm headers those define) stay in place:
// they are pre-guarded here and expand to nothing.  See include/mspmv.hpp (drop-in mode) and
// INTEGRATION.md.
#pragma once
#define MSPMV_REPLACE_REFERENCE 1
#include "mspmv.hpp"
