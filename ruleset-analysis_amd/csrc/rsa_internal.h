// Internal interface between the translation units of libruleset_hip.so (not
// part of the public C ABI in include/ruleset_hip.h).
#ifndef RSA_INTERNAL_H
#define RSA_INTERNAL_H

#include <hip/hip_runtime.h>

#include "../../include/ruleset_hip.h"

extern "C" {
// The ctx's HIP stream (every launch of a ctx goes there).
hipStream_t rsa_internal_stream(rsa_ctx* c);
// Record `msg` as the ctx's last error and return `code`.
int rsa_internal_fail(rsa_ctx* c, int code, const char* msg);
// RSA_OPT_PARSE_MODE: 0 = lines staged in LDS per workgroup, 1 = direct HBM reads,
// 2 = register-window reads (default).
int rsa_internal_parse_mode(rsa_ctx* c);
}

#endif
