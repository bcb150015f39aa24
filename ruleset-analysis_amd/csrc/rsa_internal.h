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
// The ctx's device and its bound counters (rsa_bind_counters; NULL if unbound)
// over n_rules rules.
int rsa_internal_device(rsa_ctx* c);
void rsa_internal_counters(rsa_ctx* c, unsigned long long** matches, unsigned long long** hits,
                           unsigned int** distinct, unsigned long long** thresh, uint32_t* n_rules);
// merge.hip's per-ctx state (buffers of rsa_merge), freed by rsa_ctx_destroy
// through rsa_internal_merge_free.
void** rsa_internal_merge_slot(rsa_ctx* c);
void rsa_internal_merge_free(void* state);
// RSA_OPT_ROUTE_ROWS (testing; 0 = off).
uint64_t rsa_internal_route_rows(rsa_ctx* c);
}

#endif
