// Nested per-block pauses: a thread that already holds a
// tpf::PerblockPause takes it again (the host streams' frees inside a pause,
// tpf_perblock_quiesce, tpf_host_release) without re-locking the shared mutex
// -- which throws EDEADLK ("Resource deadlock avoided") -- while other threads
// do the same.  Host only: with no server running the pauses touch no HIP call.
#include <cstdio>
#include <thread>
#include <vector>

#include "../../include/turbopfor_capi.h"
#include "../../turbopfor-cpp_amd/csrc/tpf_kernels.h"

static void nest(int depth)
{
    if (depth == 0)
    {
        tpf_perblock_quiesce();
        tpf_host_release();
        return;
    }
    const tpf::PerblockPause p;
    tpf_perblock_quiesce();
    nest(depth - 1);
}

int main()
{
    nest(4);
    std::vector<std::thread> th;
    for (int i = 0; i < 4; ++i)
        th.emplace_back([i] {
            for (int k = 0; k < 2000; ++k)
                nest((i + k) % 4);
        });
    for (std::thread & t : th)
        t.join();
    tpf_perblock_quiesce();
    std::puts("pause nesting ok");
    return 0;
}
