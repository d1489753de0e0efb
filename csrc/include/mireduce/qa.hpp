// QA protocol lines and exit status.
//
// Reference: shrQAStart / shrQAFinishExit (cuda/shared/inc/shrQATest.h:83-112,140-186,224-229):
// with --qatest print "&&&& RUNNING <exe> <args>" and "&&&& PASSED|FAILED|WAIVED <exe> <args>"
// to stderr, otherwise "[<exe>] starting..." and "[<exe>] test results...\n<STATUS>"; exit 0 for
// PASSED/WAIVED, 1 for FAILED. Difference: no 3-second exit countdown unless --countdown (bug
// B15); --prompt still waits for <Enter>.
#pragma once

namespace mireduce {

enum class QaStatus : int { Failed = 0, Passed = 1, Waived = 2 };

void qa_start(int argc, const char* const* argv);
void qa_finish(int argc, const char* const* argv, QaStatus status);
[[noreturn]] void qa_finish_exit(int argc, const char* const* argv, QaStatus status);
const char* qa_status_name(QaStatus s);

}  // namespace mireduce
