// Host check of gnss_sim_receiver_amd/csrc/exact_div.h against the host's IEEE division and fmod
// (tests/test_exact_div.py).  Modes: "div <samples per divisor>", "fmodf <stride>" (every stride-th float below
// 2^23, then every 256th up to 2^40), "fmodd <samples>" (random doubles below 2^40 and doubles next to
// multiples of 2π).  Prints "checked N mismatches M".
#define GNSSHIP_HD
#include "exact_div.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

using gnsship::div_by;
using gnsship::fmod_by;

static const double kTwoPi = 2.0 * 3.1415926535898;  // trk_loop.h kTwoPi (the reference's TWO_PI)

static bool same(double a, double b) { return std::memcmp(&a, &b, 8) == 0; }

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    long n = 0, bad = 0;
    std::mt19937_64 g(12345);
    if (!std::strcmp(argv[1], "div")) {
        const long per = argc > 2 ? std::atol(argv[2]) : 1000000;
        const double ds[] = {kTwoPi, 2e6, 4e6, 4.092e6, 5e6, 6.25e6, 8e6, 10e6, 12.5e6, 16.368e6, 20e6, 25e6, 40e6, 50e6, 100e6,
                             1575.42e6, 1561.098e6, 1176.45e6, 1207.14e6, 1227.6e6, 1602e6, 1246e6, 1268.52e6, 1278.75e6};
        for (double d : ds) {
            const double inv = 1.0 / d;
            for (long i = 0; i < per; i++) {
                const uint64_t b = g();
                const uint64_t e = 1023 - 200 + (b >> 52) % 400;
                const uint64_t bits = (b & 0x800fffffffffffffull) | (e << 52);
                double x;
                std::memcpy(&x, &bits, 8);
                n++;
                if (!same(div_by(x, d, inv), x / d)) bad++;
            }
        }
        for (long j = 0; j < per / 100 + 1; j++) {  // random divisors in [1, 2), 100 numerators each
            const uint64_t b = g(), bits = (b & 0x000fffffffffffffull) | (1023ull << 52);
            double d;
            std::memcpy(&d, &bits, 8);
            const double inv = 1.0 / d;
            for (int i = 0; i < 100; i++) {
                const uint64_t bb = g(), e = 1023 - 100 + (bb >> 52) % 200, xb = (bb & 0x800fffffffffffffull) | (e << 52);
                double x;
                std::memcpy(&x, &xb, 8);
                n++;
                if (!same(div_by(x, d, inv), x / d)) bad++;
            }
        }
        for (double z : {0.0, -0.0}) {
            n++;
            if (!same(div_by(z, 4e6, 1.0 / 4e6), z / 4e6)) bad++;
        }
    } else if (!std::strcmp(argv[1], "fmodf")) {
        const uint32_t stride = argc > 2 ? static_cast<uint32_t>(std::atol(argv[2])) : 1u;
        const double inv = 1.0 / kTwoPi;
        for (uint32_t u = 0; u < 0x53800000u; u += (u < 0x4b000000u ? stride : 256u)) {  // |x| < 2^40
            for (uint32_t s : {0u, 0x80000000u}) {
                const uint32_t ub = u | s;
                float f;
                std::memcpy(&f, &ub, 4);
                const double x = f;
                n++;
                if (!same(fmod_by(x, kTwoPi, inv), std::fmod(x, kTwoPi))) bad++;
            }
        }
    } else if (!std::strcmp(argv[1], "fmodd")) {
        const long cnt = argc > 2 ? std::atol(argv[2]) : 1000000;
        const double inv = 1.0 / kTwoPi;
        for (long i = 0; i < cnt; i++) {
            const uint64_t b = g(), e = 1023 - 60 + (b >> 52) % 100, xb = (b & 0x800fffffffffffffull) | (e << 52);
            double x;
            std::memcpy(&x, &xb, 8);
            n++;
            if (!same(fmod_by(x, kTwoPi, inv), std::fmod(x, kTwoPi))) bad++;
        }
        for (long k = -200000; k <= 200000; k++)
            for (int d = -3; d <= 3; d++) {
                double x = static_cast<double>(k) * kTwoPi;
                for (int j = 0; j < (d < 0 ? -d : d); j++) x = std::nextafter(x, d < 0 ? -1e300 : 1e300);
                n++;
                if (!same(fmod_by(x, kTwoPi, inv), std::fmod(x, kTwoPi))) bad++;
            }
        for (double x : {1e15, -3e20, 0x1p40, -0x1p40, 1.0 / 0.0, 0.0, -0.0}) {
            n++;
            const double a = fmod_by(x, kTwoPi, inv), r = std::fmod(x, kTwoPi);
            if (!same(a, r) && !(a != a && r != r)) bad++;
        }
    } else {
        return 2;
    }
    std::printf("checked %ld mismatches %ld\n", n, bad);
    return bad ? 1 : 0;
}
