// Host helpers shared by the C-ABI entry points (not exported).
#pragma once
#include <cstdint>

struct phip_handle;

namespace phip_host {

// The stream every call of the handle runs on (its own or phip_set_stream's)
// and its device: the shard group (phip_group.hip) queues its RCCL calls there.
void* handle_stream(phip_handle* h);
int handle_device(const phip_handle* h);

// A timed region on the handle's stream (HIP events, like the engine's own
// kernels; nothing when timing is off): the group's RCCL calls show up in
// phip_last_timings under `name`.  timing_end takes what timing_begin gave.
void* timing_begin(phip_handle* h, const char* name);
void timing_end(phip_handle* h, void* token);

// The request parsing of API.takeBucket (api.go:55-65): the name-length check
// (returns 400 with ErrNameTooLarge's text as the body), ParseRate with its
// error ignored (the Rate Go returns beside the error), count 0 / error -> 1.
// Returns 0 when the Take should run.
int api_prepare(const uint8_t* name, uint32_t len, const char* rate, uint32_t rate_len,
                const char* count, uint32_t count_len, int64_t* freq, int64_t* per, uint64_t* n,
                char* body, uint32_t* body_len);

}  // namespace phip_host
