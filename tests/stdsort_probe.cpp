// Test helper (tests/test_aten_argsort.py): the permutation libstdc++'s std::sort (or
// std::partial_sort over the whole range: the introsort's depth-limit fallback) gives a vector of
// (float value, index) pairs under the descending comparator of ATen's CPU sort kernel
// (KeyValueCompDesc: NaN first, then larger values first). Built with g++ at test time.
//   stdin: "<sort|partial> <n>\n" then n values as C99 hex floats; stdout: the n indices.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

int main() {
    char mode[16] = {0};
    long n = 0;
    if (std::scanf("%15s %ld", mode, &n) != 2 || n < 0) return 2;
    std::vector<std::pair<float, long>> v(static_cast<size_t>(n));
    char tok[64];
    for (long i = 0; i < n; ++i) {
        if (std::scanf("%63s", tok) != 1) return 3;
        v[static_cast<size_t>(i)] = {std::strtof(tok, nullptr), i};
    }
    auto desc = [](const std::pair<float, long>& a, const std::pair<float, long>& b) {
        return (std::isnan(a.first) && !std::isnan(b.first)) || a.first > b.first;
    };
    if (std::strcmp(mode, "partial") == 0) std::partial_sort(v.begin(), v.end(), v.end(), desc);
    else std::sort(v.begin(), v.end(), desc);
    for (const auto& p : v) std::printf("%ld\n", p.second);
    return 0;
}
