// glibc_sincosf_check — pins gnss_sim_receiver_amd/csrc/glibc_sincosf.h (the device's phasor trig)
// and glibc_atanf.h (the loop's discriminators) against this host's own glibc sinf / cosf / sincosf /
// atanf / atan2f, bit for bit.  Test infrastructure: built and
// run by tests/test_glibc_sincosf.py (compiled for the host with -ffp-contract=off, as the device
// code is built).
//
//   glibc_sincosf_check range LO_BITS HI_BITS      every float whose bit pattern lies in [LO, HI)
//   glibc_sincosf_check random COUNT SEED          COUNT random bit patterns (the whole float line)
//   glibc_sincosf_check uniform COUNT SEED LO HI   COUNT floats uniform in [LO, HI)
//   glibc_sincosf_check fma                        1 if the CPU has FMA (glibc then runs its FMA build)
//   FN=atan (environment): the same modes for atanf, and atan2f(x, 1 / x), atan2f(x, −x), atan2f(−x, y)
//                                                  with y the next random draw
//   FN=log: the same modes for logf and log10f (glibc_logf.h)
// Prints "checked N mismatches M" (and the first few mismatching arguments); exit 0 iff M == 0.
#define GNSSHIP_HD
#include "../../gnss_sim_receiver_amd/csrc/glibc_sincosf.h"
#include "../../gnss_sim_receiver_amd/csrc/glibc_atanf.h"
#include "../../gnss_sim_receiver_amd/csrc/glibc_logf.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>
#include <atomic>

#include <cpuid.h>

extern "C" void sincosf(float, float*, float*);

namespace {

std::atomic<uint64_t> g_bad{0};
std::atomic<int> g_printed{0};

bool same(float a, float b) { return std::memcmp(&a, &b, 4) == 0 || (std::isnan(a) && std::isnan(b)); }

bool g_atan = false, g_log = false;

void check_log(float x)
{
    const float a = gnsship::glibc_logf(x), ha = ::logf(x);
    const float b = gnsship::glibc_log10f(x), hb = ::log10f(x);
    if (!same(a, ha) || !same(b, hb)) {
        g_bad++;
        if (g_printed++ < 8) std::printf("mismatch x=%a: logf %a/%a log10f %a/%a\n", x, a, ha, b, hb);
    }
}

void check_atan(float x, float y)
{
    const float a = gnsship::glibc_atanf(x), ha = ::atanf(x);
    const float b = gnsship::glibc_atan2f(x, y), hb = ::atan2f(x, y);
    const float c = gnsship::glibc_atan2f(y, -x), hc = ::atan2f(y, -x);
    if (!same(a, ha) || !same(b, hb) || !same(c, hc)) {
        g_bad++;
        if (g_printed++ < 8)
            std::printf("mismatch x=%a y=%a: atanf %a/%a atan2f(x,y) %a/%a atan2f(y,-x) %a/%a\n", x, y, a, ha, b, hb, c, hc);
    }
}

void check_one(float x)
{
    if (g_log) {
        check_log(x);
        return;
    }
    if (g_atan) {
        const uint32_t h = __builtin_bit_cast(uint32_t, x) * 2654435761u;
        check_atan(x, __builtin_bit_cast(float, (h & 0x807fffffu) | (__builtin_bit_cast(uint32_t, x) & 0x7f800000u) ^ ((h >> 8) & 0x07800000u)));
        return;
    }
    float s, c;
    gnsship::glibc_sincosf(x, &s, &c);
    const float hs = ::sinf(x), hc = ::cosf(x);
    float ss, sc;
    ::sincosf(x, &ss, &sc);
    if (!same(s, hs) || !same(c, hc) || !same(ss, hs) || !same(sc, hc)) {
        g_bad++;
        if (g_printed++ < 8)
            std::printf("mismatch x=%a: dev (%a, %a) sinf/cosf (%a, %a) sincosf (%a, %a)\n", x, s, c, hs, hc, ss, sc);
    }
}

template <class F>
void parallel(uint64_t n, F f)
{
    const unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([=] {
            for (uint64_t i = t; i < n; i += nt) f(i);
        });
    for (auto& x : th) x.join();
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    if (const char* f = std::getenv("FN")) {
        g_atan = !std::strcmp(f, "atan");
        g_log = !std::strcmp(f, "log");
    }
    const char* mode = argv[1];
    uint64_t n = 0;
    if (!std::strcmp(mode, "fma")) {
        unsigned a, b, c, d;
        __get_cpuid(1, &a, &b, &c, &d);
        std::printf("%d\n", (c >> 12) & 1);
        return 0;
    } else if (!std::strcmp(mode, "range") && argc >= 4) {
        const uint64_t lo = std::strtoull(argv[2], nullptr, 0), hi = std::strtoull(argv[3], nullptr, 0);
        n = hi - lo;
        parallel(n, [=](uint64_t i) { check_one(__builtin_bit_cast(float, static_cast<uint32_t>(lo + i))); });
    } else if (!std::strcmp(mode, "random") && argc >= 4) {
        n = std::strtoull(argv[2], nullptr, 0);
        const uint64_t seed = std::strtoull(argv[3], nullptr, 0);
        parallel(n, [=](uint64_t i) {
            std::mt19937_64 g(seed ^ (i * 0x9E3779B97F4A7C15ull));
            check_one(__builtin_bit_cast(float, static_cast<uint32_t>(g())));
        });
    } else if (!std::strcmp(mode, "uniform") && argc >= 6) {
        n = std::strtoull(argv[2], nullptr, 0);
        const uint64_t seed = std::strtoull(argv[3], nullptr, 0);
        const double lo = std::atof(argv[4]), hi = std::atof(argv[5]);
        parallel(n, [=](uint64_t i) {
            std::mt19937_64 g(seed ^ (i * 0x9E3779B97F4A7C15ull));
            const double u = static_cast<double>(g() >> 11) * 0x1p-53;
            check_one(static_cast<float>(lo + (hi - lo) * u));
        });
    } else {
        return 2;
    }
    std::printf("checked %llu mismatches %llu\n", static_cast<unsigned long long>(n), static_cast<unsigned long long>(g_bad.load()));
    return g_bad.load() == 0 ? 0 : 1;
}
