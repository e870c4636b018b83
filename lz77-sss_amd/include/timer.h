// timer.h -- hipEvent phase timer shared by the pos_t = uint32_t and uint64_t engines.
#pragma once
#include "lz77sss_internal.h"

#include <cstdlib>
#include <string>
#include <utility>
#include <vector>

namespace lz {

// (held / peak count the device allocations of every session in the process: g_dev_bytes and
// g_phase_peak are process-wide, lz77sss.h lz77sss_session_phase_mem)
struct phase_mem {
    uint64_t held = 0;      // device bytes of the process's buffers when the phase was enqueued
    uint64_t peak = 0;      // their peak during the phase
    uint64_t hbm_free = 0;  // free device memory then (hipMemGetInfo: the whole GPU)
};
struct phase_timer {
    hipStream_t st = nullptr;
    std::vector<std::pair<std::string, hipEvent_t>> marks;
    std::vector<phase_mem> mem;  // per mark (the allocations are host-side: exact at enqueue time)
    std::vector<hipEvent_t> pool;  // events are reused across calls (created once)
    size_t used = 0;
    void begin(hipStream_t s) {
        st = s;
        clear();
        mark("start");
    }
    void mark(const char* name) {
        if (used == pool.size()) {
            hipEvent_t e;
            LZ_HIP(hipEventCreate(&e));
            pool.push_back(e);
        }
        hipEvent_t e = pool[used++];
        LZ_HIP(hipEventRecord(e, st));
        marks.emplace_back(name, e);
        phase_mem m;
        m.held = g_dev_bytes.load();
        m.peak = g_phase_peak.exchange(m.held);
        if (m.peak < m.held) m.peak = m.held;
        // the driver's free-memory query is a host call between phases: once per call (at the start
        // mark), later marks derive it from this process's own allocations since then, unless
        // LZ77SSS_PHASE_MEM asks for a query at every mark
        static const bool query_all = std::getenv("LZ77SSS_PHASE_MEM") != nullptr;
        if (mem.empty() || query_all) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess) m.hbm_free = fr;
        } else {
            const phase_mem& m0 = mem.front();
            m.hbm_free = m0.hbm_free + m0.held >= m.held ? m0.hbm_free + m0.held - m.held : 0;
        }
        mem.push_back(m);
    }
    void clear() {
        marks.clear();
        mem.clear();
        used = 0;
    }
    // (name, ms since previous mark)
    std::vector<std::pair<std::string, double>> read() {
        std::vector<std::pair<std::string, double>> out;
        if (marks.empty()) return out;
        LZ_HIP(hipEventSynchronize(marks.back().second));
        for (size_t i = 1; i < marks.size(); i++) {
            float ms = 0;
            LZ_HIP(hipEventElapsedTime(&ms, marks[i - 1].second, marks[i].second));
            out.emplace_back(marks[i].first, ms);
        }
        return out;
    }
    ~phase_timer() {
        for (auto& e : pool) (void)hipEventDestroy(e);
    }
};

}  // namespace lz
