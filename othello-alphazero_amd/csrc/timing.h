// Host-side timing arithmetic of the engine (capi.hip), kept in a header of
// its own so the CPU tests compile it with g++ (tests/test_cpu_bench.py).
#pragma once

#include <algorithm>
#include <utility>
#include <vector>

// Total length covered by a set of [begin, end] intervals (any sign: they
// may be measured from one group's first event, and another pipeline group's
// stream may run ahead of it). The ResNet launches of different NN chains
// overlap; their union is the time some launch ran. The engine passes int64
// clock ticks (exact over any window; ADVICE r4: float ms lost 0.01-0.06 ms of
// resolution over minutes-long windows) and converts the sum once.
template <typename T>
inline double interval_union(std::vector<std::pair<T, T>>& iv) {
    std::sort(iv.begin(), iv.end());
    double sum = 0.0;
    bool open = false;
    T lo = T(0), hi = T(0);
    for (const auto& x : iv) {
        if (!open || x.first > hi) {
            if (open) sum += (double)hi - lo;
            lo = x.first;
            hi = x.second;
            open = true;
        } else if (x.second > hi) {
            hi = x.second;
        }
    }
    if (open) sum += (double)hi - lo;
    return sum;
}
