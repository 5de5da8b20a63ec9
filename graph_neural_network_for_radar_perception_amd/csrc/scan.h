#pragma once
#include <hip/hip_runtime.h>

namespace rg {
// out[0..n] = exclusive prefix sum of in[0..n) with out[n] = total; total also
// written to *total_out when non-null.  ws must hold scan_workspace_bytes(n).
size_t scan_workspace_bytes(long n);
int exclusive_scan(const int* in, long n, int* out, int* total_out, void* ws, hipStream_t st);
}  // namespace rg
