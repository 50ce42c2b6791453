// adjust_mmba.h -- mmSolver plug-in side of the MI355X bundle-adjustment
// core (libmmba.so, include/mmba.h).  Drop-in for the two cminpack calls of
// solveFrames (src/mmSolver/adjust/adjust_base.cpp:1175-1184); see
// INTEGRATION.md for the three lines that dispatch to it.
//
// This file and adjust_mmba.cpp (the Maya layer: scene reads through the
// reference's Maya helpers) belong in src/mmSolver/adjust/ of the mmSolver
// tree and build with the plug-in (Maya SDK).  Everything below the reads --
// SolverData -> mmba_problem, the plan cache, the solve, the result mapping --
// is adjust_mmba_core.{h,cpp}, which has no Maya dependency and is built and
// tested in this repository (tests/shim, tests/test_shim_core.py).
#ifndef MM_SOLVER_CORE_BUNDLE_ADJUST_MMBA_H
#define MM_SOLVER_CORE_BUNDLE_ADJUST_MMBA_H

#include <vector>

#include "adjust_data.h"
#include "adjust_results.h"

// Same signature and contract as solve_3d_cminpack_lmder
// (adjust_cminpack_lmder.cpp:64-198): paramList in = x0 (internal), out =
// the solved x; errorList, userData.errorList and
// userData.errorDistanceList hold what the last measureErrors left (stale
// Jacobian columns included).  The LM variant follows
// solverOptions.solverType (lmder or lmdif semantics).  Returns false when
// the device cannot run this solve (no gfx950 device, a scene the core does
// not map): the caller then runs the cminpack function instead.
bool solve_3d_mmba(SolverOptions &solverOptions, int numberOfParameters,
                   int numberOfErrors, std::vector<double> &paramList,
                   std::vector<double> &errorList,
                   std::vector<double> &paramWeightList, SolverData &userData,
                   SolverResult &solveResult);

// FrameSolveMode::kPerFrame (adjust_base.cpp:1430-1484) in one device call
// when no static attribute is solved: userData / paramList / errorList are
// prepared ONCE for all frames (as solveFrames prepares an all-frames
// solve), every frame is solved by its own lmder/lmdif in one launch
// (mmba_plan_solve_per_frame), perFrameResults[i] receives frame i's
// SolverResult and paramList the values each frame's solveFrames would
// write back.  Returns false when the frames are not independent (a static
// parameter chains them) or the device cannot run it; the caller then keeps
// the reference per-frame loop.
bool solve_frames_mmba_per_frame(SolverOptions &solverOptions,
                                 std::vector<double> &paramList,
                                 std::vector<double> &paramWeightList,
                                 SolverData &userData,
                                 std::vector<SolverResult> &perFrameResults);

// Drops the cached device context and plans (plug-in unload).
void mmba_shim_release();

#endif  // MM_SOLVER_CORE_BUNDLE_ADJUST_MMBA_H
