// Host helpers shared by the C-ABI entry points (not exported).
#pragma once
#include <cstdint>

#include "patrolhip.h"

namespace phip_host {

// The stream every call of the handle runs on (its own or phip_set_stream's)
// and its device: the shard group (phip_group.hip) queues its RCCL calls there.
void* handle_stream(phip_handle* h);
int handle_device(const phip_handle* h);

// Owner routing as phip_route_pack does it, queued on `stream` (a hipStream_t
// of the handle's device) with no host synchronisation: the pipelined
// exchange of phip_group_receive packs chunk k+1 while chunk k travels.
//   route_dir:  the sender-side combine's hot-name directory, from a strided
//               sample of the whole batch m (nullptr below kRouteMinBatch);
//   route_pack: the stable owner partition of m (one chunk) into owner-major
//               send buffers, with the per-owner totals in counts / nbytes
//               (device), combining with `dir` when it is not null.
// The scratch they use is the handle's, reused in stream order: every pack
// of one call must be queued on the same stream, none larger than the first.
int route_dir(phip_handle* h, void* stream, const phip_msgs* m, uint32_t world, const void** dir);
int route_pack(phip_handle* h, void* stream, const phip_msgs* m, uint32_t world, const void* dir,
               uint8_t* names, uint32_t* lens, uint64_t* a, uint64_t* t, int64_t* e,
               uint64_t* counts, uint64_t* nbytes);
const char* last_error(phip_handle* h);

// The request parsing of API.takeBucket (api.go:55-65): the name-length check
// (returns 400 with ErrNameTooLarge's text as the body), ParseRate with its
// error ignored (the Rate Go returns beside the error), count 0 / error -> 1.
// Returns 0 when the Take should run.
int api_prepare(const uint8_t* name, uint32_t len, const char* rate, uint32_t rate_len,
                const char* count, uint32_t count_len, int64_t* freq, int64_t* per, uint64_t* n,
                char* body, uint32_t* body_len);

}  // namespace phip_host
