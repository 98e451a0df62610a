// Exhaustive check of core/detmath.h against this machine's glibc: every one of the 2^32 float
// inputs of sin, cos, sincos, exp, log, asin, acos, atan, tan, expm1 and sinh, and 10^8 sampled
// (y, x) pairs of atan2 (random bit patterns, ratios near 1, and |y/x| spread over 2^+-30).
//   g++ -O2 -std=c++17 -ffp-contract=off -pthread -I pbrt-v4_amd/csrc tools/detmath_exhaustive.cpp
// Prints one line per function with the mismatch count; exit status 1 if any is nonzero.
// The last run's output is kept in profiles/r06_detmath_exhaustive.txt.
#include "core/detmath.h"

#include <atomic>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

using namespace pbrt_amd;

static bool Same(float a, float b) { return detm::Bits(a) == detm::Bits(b) || (a != a && b != b); }

template <class G, class C>
static long Exhaustive(const char *name, G g, C c) {
    std::atomic<long> bad{0};
    std::atomic<int> shown{0};
    const unsigned T = std::max(1u, std::thread::hardware_concurrency());
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            long b = 0;
            for (uint64_t u = t; u < (1ull << 32); u += T) {
                const float x = detm::FromBits((uint32_t)u);
                const float a = g(x), d = c(x);
                if (!Same(a, d)) {
                    ++b;
                    if (shown.fetch_add(1) < 4) printf("  %s(%a): glibc %a, detmath %a\n", name, x, a, d);
                }
            }
            bad += b;
        });
    for (auto &x : th) x.join();
    printf("%-8s %ld mismatches of 4294967296\n", name, bad.load());
    fflush(stdout);
    return bad.load();
}

int main() {
    long bad = 0;
    bad += Exhaustive("sin", [](float x) { return sinf(x); }, detm::Sin);
    bad += Exhaustive("cos", [](float x) { return cosf(x); }, detm::Cos);
    bad += Exhaustive("sincos", [](float x) { float s, c; sincosf(x, &s, &c); return s + 2.f * c; },
                      [](float x) { float s, c; detm::SinCos(x, &s, &c); return s + 2.f * c; });
    bad += Exhaustive("exp", [](float x) { return expf(x); }, detm::Exp);
    bad += Exhaustive("log", [](float x) { return logf(x); }, detm::Log);
    bad += Exhaustive("asin", [](float x) { return asinf(x); }, detm::ASin);
    bad += Exhaustive("acos", [](float x) { return acosf(x); }, detm::ACos);
    bad += Exhaustive("atan", [](float x) { return atanf(x); }, detm::ATan);
    bad += Exhaustive("tan", [](float x) { return tanf(x); }, detm::Tan);
    bad += Exhaustive("expm1", [](float x) { return expm1f(x); }, detm::Expm1);
    bad += Exhaustive("sinh", [](float x) { return sinhf(x); }, detm::Sinh);
    std::mt19937 g(1);
    std::uniform_real_distribution<float> U(-10, 10);
    long b2 = 0, n = 0;
    for (int i = 0; i < 100000000; ++i) {
        float y, x;
        if (i % 3 == 0) {
            y = detm::FromBits(g());
            x = detm::FromBits(g());
        } else {
            y = U(g);
            x = U(g);
            if (i % 3 == 2) x = ldexpf(x, (int)(g() % 61) - 30);
        }
        ++n;
        if (!Same(atan2f(y, x), detm::ATan2(y, x))) {
            if (b2 < 4) printf("  atan2(%a, %a): glibc %a, detmath %a\n", y, x, atan2f(y, x), detm::ATan2(y, x));
            ++b2;
        }
    }
    printf("%-8s %ld mismatches of %ld sampled pairs\n", "atan2", b2, n);
    return bad + b2 ? 1 : 0;
}
