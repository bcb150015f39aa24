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
// RSA_OPT_PARSE_STAGED: the mapper-form parse stages each workgroup's lines in
// LDS (k_parse) instead of the register-window reads (k_parse_win, default).
int rsa_internal_parse_staged(rsa_ctx* c);
}

#endif
