// Host-side timing arithmetic of the engine (capi.hip), kept in a header of
// its own so the CPU tests compile it with g++ (tests/test_cpu_bench.py).
#pragma once

#include <algorithm>
#include <utility>
#include <vector>

// Total length covered by a set of [begin, end] intervals (ms, any sign:
// they are measured from one group's first event, and another pipeline
// group's stream may run ahead of it). The ResNet launches of different NN
// chains overlap; their union is the time some launch ran.
inline double interval_union(std::vector<std::pair<float, float>>& iv) {
    std::sort(iv.begin(), iv.end());
    double sum = 0.0;
    bool open = false;
    float lo = 0.0f, hi = 0.0f;
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
