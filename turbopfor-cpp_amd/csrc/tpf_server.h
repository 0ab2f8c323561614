// tpf_server.h -- mailbox layout of the per-block block server (shared by
// p4_server.hip and host_api.cpp; internal).
//
// The per-block drop-in calls (include/turbopfor.h, one block per call) are
// served by a resident kernel that polls mailboxes, instead of one kernel
// launch plus one stream synchronise per call.
// Each mailbox has two halves:
//   ServerReq (host -> device): request line + input payload.  Placed in
//     fine-grained DEVICE memory that the host writes through the BAR, so the
//     kernel polls and stages from its own HBM instead of reading across PCIe
//     (tpf_perblock_mode 0; mode 2 keeps it in coherent pinned host memory).
//   ServerAns (device -> host): answer line + output payload, always in
//     coherent pinned host memory, so the host polls its own cache.
// Host and device exchange only plain loads/stores ordered by fences -- no
// atomics on shared memory:
//   host  : payload and request fields, release (+ sfence), req = r
//   device: sees req != last, acquire, serves, release, ack = r
//   host  : sees ack == r, acquire, reads the result
// The kernel raises ServerAns::alive while it runs (the host posts without
// querying the launch's event) and exits once every mailbox of the launch has
// been idle for kServerIdleTicks of the 100 MHz real-time clock (or at once
// when told to stop); the host sees alive drop / the launch complete and
// relaunches it on the next request.
#pragma once

#include <stdint.h>

namespace tpf
{

// One wave per mailbox, four per workgroup.  Round 5: sixteen workgroups
// (64 mailboxes: 64 threads call concurrently) instead of one (4 mailboxes:
// a fifth calling thread waited for a free one).  The launch's
// workgroups share one device-side control word set (ServerCtl) so they leave
// together.
constexpr uint32_t kServerWavesPerWG = 4;
constexpr uint32_t kServerWGs = 16;
constexpr uint32_t kServerBoxes = kServerWavesPerWG * kServerWGs;
constexpr uint32_t kServerPayload = 8192;      // bytes in / out per request
constexpr uint64_t kServerIdleTicks = 1000000; // 10 ms of s_memrealtime (100 MHz)
// A launch also leaves after serving for 5 ms, busy or not (the next call
// relaunches it, ~20 us per 5 ms of traffic): hipDeviceSynchronize -- e.g.
// torch.cuda.synchronize() in another thread -- waits for every stream of the
// device, the server's included, and under back-to-back per-block calls an
// unbounded launch never idled out, so such a wait never returned (round 4,
// scripts/graph_canary.py with a per-block caller thread).
constexpr uint64_t kServerMaxTicks = 500000;

enum : uint32_t
{
    kOpDec = 0,
    kOpEnc = 1,
};

// The request fields share ONE 64-byte line with the request number: the
// host writes the fields, then (release) req; the device polls the line's
// first 8 words with one 8-lane dword load (one read of the line, which
// returns it as one unit), so a new req arrives with its fields.
struct alignas(128) ServerReqBox
{
    uint32_t req;     // request number (monotonic, 0 = none yet)
    uint32_t op;      // kOpDec / kOpEnc
    uint32_t fmt;     // TPF_FMT_*
    uint32_t n;       // values per call
    uint32_t d1;      // delta-1 variant
    uint32_t in_len;  // decode: block bytes; encode: value bytes
    uint32_t start_lo, start_hi; // D1 start
    uint32_t pad0[24];
    uint8_t in[kServerPayload];
};

struct alignas(128) ServerAnsBox
{
    uint32_t ack;     // last request served
    uint32_t result;  // decode: bytes consumed; encode: bytes produced; 0xFFFFFFFF = malformed
    uint32_t written; // decode: values written
    uint32_t pad1[29];
    uint8_t out[kServerPayload];
};

struct alignas(128) ServerReq
{
    uint32_t stop; // host -> device: exit now
    uint32_t pad[31];
    ServerReqBox box[kServerBoxes];
};

// Device memory (coarse-grained, zeroed before every launch): what the
// launch's workgroups share.
struct alignas(128) ServerCtl
{
    unsigned long long last_active; // s_memrealtime of the latest request served (or workgroup start)
    uint32_t quit;                  // one workgroup decided to leave: the others follow
    uint32_t live;                  // workgroups still serving; the last to leave lowers ServerAns::alive
};

struct alignas(128) ServerAns
{
    uint32_t alive; // device -> host: 1 while a launch is serving
    uint32_t pad[31];
    ServerAnsBox box[kServerBoxes];
};

} // namespace tpf
