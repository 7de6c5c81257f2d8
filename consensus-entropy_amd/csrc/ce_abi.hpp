// ce_abi.hpp -- error reporting shared by the translation units of libce_amd.so
// (ce_kernels.hip defines them; ce_xgb.hip uses them).  Hidden: not part of
// the exported C-ABI.
#pragma once
#define CE_HIDDEN __attribute__((visibility("hidden")))

CE_HIDDEN int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
CE_HIDDEN int check_launch(const char* what);
// the kernel the last selection on this thread launched for its main pass, in
// the demangled form rocprofv3 reports (ce_last_kernel(); "" = none noted)
CE_HIDDEN void note_kernel(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
