// codes.cpp — product-side PRN replica generators (host C++), exported through the C ABI so the
// adapters can build the local codes they hand to the correlator / acquisition engines.
//
//  GPS L1 C/A   : G1 = 1 + x^3 + x^10, G2 = 1 + x^2 + x^3 + x^6 + x^8 + x^9 + x^10, PRN code =
//                 G1 ⊕ G2 delayed by the IS-GPS-200 delay  (reference gps_sdr_signal_replica.cc:25-110)
//  BeiDou B1I   : 11-stage Gold code, G2 output taps per PRN  (beidou_b1i_signal_replica.cc:26-110)
//  sampled forms: the Borre-style upsampling with a float chip clock and the last sample forced
//                 to the last chip  (gps_sdr_signal_replica.cc:145-185, beidou_b1i_signal_replica.cc:142-180)
//
// Registers are kept as integers (bit i = register cell i) instead of bitsets; outputs are identical,
// which tests/test_codes.py checks against the oracle and the golden fixtures.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "gnsship.h"

namespace {

// IS-GPS-200 G2 delays (chips) for PRN 1..210 (same table the reference carries at :41-51).
constexpr int16_t kGpsG2Delay[210] = {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470, 471, 472, 473, 474,
    509, 512, 513, 514, 515, 516, 859, 860, 861, 862, 863, 950, 947, 948, 950, 67, 103, 91, 19, 679, 225, 625, 946, 638, 161, 1001, 554,
    280, 710, 709, 775, 864, 558, 220, 397, 55, 898, 759, 367, 299, 1018, 729, 695, 780, 801, 788, 732, 34, 320, 327, 389, 407, 525, 405,
    221, 761, 260, 326, 955, 653, 699, 422, 188, 438, 959, 539, 879, 677, 586, 153, 792, 814, 446, 264, 1015, 278, 536, 819, 156, 957,
    159, 712, 885, 461, 248, 713, 126, 807, 279, 122, 197, 693, 632, 771, 467, 647, 203, 145, 175, 52, 21, 237, 235, 886, 657, 634, 762,
    355, 1012, 176, 603, 130, 359, 595, 68, 386, 797, 456, 499, 883, 307, 127, 211, 121, 118, 163, 628, 853, 484, 289, 811, 202, 1021,
    463, 568, 904, 670, 230, 911, 684, 309, 644, 932, 12, 314, 891, 212, 185, 675, 503, 150, 395, 345, 846, 798, 992, 357, 995, 877, 112,
    144, 476, 193, 109, 445, 291, 87, 399, 292, 901, 339, 208, 711, 189, 263, 537, 663, 942, 173, 900, 30, 500, 935, 556, 373, 85, 652, 310};

// Output sequence of a Fibonacci LFSR: state bit i is register cell i, cell 0 is the output and
// the register shifts towards cell 0; `fb_mask` selects the cells XORed into the new last cell.
template <int STAGES>
void lfsr_sequence(uint32_t state, uint32_t fb_mask, int len, uint8_t* out)
{
    for (int i = 0; i < len; i++) {
        out[i] = state & 1u;
        const uint32_t fb = __builtin_parity(state & fb_mask);
        state = (state >> 1) | (fb << (STAGES - 1));
    }
}

// BeiDou B1I G2 phase-selector taps (ICD stage numbers, stage k ↔ register cell 11-k; 0 = unused), PRN 1..63.
constexpr uint8_t kB1iTap[63][3] = {{1, 3, 0}, {1, 4, 0}, {1, 5, 0}, {1, 6, 0}, {1, 8, 0}, {1, 9, 0}, {1, 10, 0}, {1, 11, 0}, {2, 7, 0},
    {3, 4, 0}, {3, 5, 0}, {3, 6, 0}, {3, 8, 0}, {3, 9, 0}, {3, 10, 0}, {3, 11, 0}, {4, 5, 0}, {4, 6, 0}, {4, 8, 0}, {4, 9, 0}, {4, 10, 0},
    {4, 11, 0}, {5, 6, 0}, {5, 8, 0}, {5, 9, 0}, {5, 10, 0}, {5, 11, 0}, {6, 8, 0}, {6, 9, 0}, {6, 10, 0}, {6, 11, 0}, {8, 9, 0},
    {8, 10, 0}, {8, 11, 0}, {9, 10, 0}, {9, 11, 0}, {10, 11, 0}, {2, 7, 1}, {3, 4, 1}, {3, 6, 1}, {3, 8, 1}, {3, 10, 1}, {3, 11, 1},
    {4, 5, 1}, {4, 9, 1}, {5, 6, 1}, {5, 8, 1}, {5, 10, 1}, {5, 11, 1}, {6, 9, 1}, {8, 9, 1}, {9, 10, 1}, {9, 11, 1}, {3, 7, 2},
    {5, 7, 2}, {7, 9, 2}, {4, 5, 3}, {4, 9, 3}, {5, 6, 3}, {5, 8, 3}, {5, 10, 3}, {5, 11, 3}, {6, 9, 3}};

int gps_chips(int32_t prn, uint32_t chip_shift, int8_t* chips)
{
    if (prn < 1 || prn > 210) return GNSSHIP_E_INVAL;
    constexpr int L = 1023;
    uint8_t g1[L], g2[L];
    // cell i ↔ polynomial stage 10-i: G1 taps x^3,x^10 → cells 7,0; G2 taps x^2,x^3,x^6,x^8,x^9,x^10
    // → cells 8,7,4,2,1,0.  All-ones initial state.
    lfsr_sequence<10>(0x3FFu, (1u << 0) | (1u << 7), L, g1);
    lfsr_sequence<10>(0x3FFu, (1u << 0) | (1u << 1) | (1u << 2) | (1u << 4) | (1u << 7) | (1u << 8), L, g2);
    uint32_t d = (static_cast<uint32_t>(L - kGpsG2Delay[prn - 1]) + chip_shift) % L;
    for (int i = 0; i < L; i++) {
        chips[i] = (g1[(i + chip_shift) % L] ^ g2[d]) ? 1 : -1;
        d = (d + 1) % L;
    }
    return GNSSHIP_OK;
}

int b1i_chips(int32_t prn, uint32_t chip_shift, int8_t* chips)
{
    if (prn < 1 || prn > 63) return GNSSHIP_E_INVAL;
    constexpr int L = 2046;
    // initial phase 01010101010 (cell 0 = rightmost character of the string)
    constexpr uint32_t init = 0x2AAu;
    uint8_t g1[L], g2[L];
    lfsr_sequence<11>(init, 0x41Fu /* cells 0-4,10 */, L, g1);
    // G2: output = XOR of the selected stages of the current state; feedback cells 0,2,3,6,7,8,9,10
    uint32_t s = init;
    const uint8_t* tap = kB1iTap[prn - 1];
    for (int i = 0; i < L; i++) {
        uint32_t o = ((s >> (11 - tap[0])) ^ (s >> (11 - tap[1]))) & 1u;
        if (tap[2]) o ^= (s >> (11 - tap[2])) & 1u;
        g2[i] = static_cast<uint8_t>(o);
        const uint32_t fb = __builtin_parity(s & 0x7CDu);
        s = (s >> 1) | (fb << 10);
    }
    uint32_t d = chip_shift % L;
    for (int i = 0; i < L; i++) {
        chips[i] = (g1[(i + chip_shift) % L] ^ g2[d]) ? 1 : -1;
        d = (d + 1) % L;
    }
    return GNSSHIP_OK;
}

// Borre upsampling (float chip clock), code value placed in re (imag_part=false) or im.
// tc_double_div: the B1I generator forms the chip period as 1.0 / float (a double division,
// beidou_b1i_signal_replica.cc:146), the GPS one as 1.0F / float (gps_sdr_signal_replica.cc:150).
int sample_code(const int8_t* chips, int code_len, int32_t chip_rate, int32_t fs, bool imag_part, bool tc_double_div, float* dest)
{
    if (fs <= 0) return GNSSHIP_E_INVAL;
    const float tc = tc_double_div ? static_cast<float>(1.0 / static_cast<double>(static_cast<float>(chip_rate)))
                                   : 1.0F / static_cast<float>(chip_rate);
    const float ts = 1.0F / static_cast<float>(fs);
    const auto n = static_cast<int32_t>(static_cast<double>(fs) / (static_cast<double>(chip_rate) / static_cast<double>(code_len)));
    for (int32_t i = 0; i < n; i++) {
        const float aux = (ts * (static_cast<float>(i) + 1)) / tc;
        int32_t k = static_cast<int32_t>(static_cast<int64_t>(aux + 1)) - 1;
        if (i == n - 1) k = code_len - 1;
        const float v = static_cast<float>(chips[k]);
        dest[2 * i] = imag_part ? 0.0F : v;
        dest[2 * i + 1] = imag_part ? v : 0.0F;
    }
    return n;
}

}  // namespace

extern "C" int gnsship_gps_l1_ca_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift)
{
    if (!dest) return GNSSHIP_E_INVAL;
    int8_t c[1023];
    if (int rc = gps_chips(prn, chip_shift, c)) return rc;
    for (int i = 0; i < 1023; i++) dest[i] = static_cast<float>(c[i]);
    return GNSSHIP_OK;
}

extern "C" int gnsship_gps_l1_ca_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t fs, uint32_t chip_shift)
{
    if (!dest) return GNSSHIP_E_INVAL;
    int8_t c[1023];
    if (int rc = gps_chips(static_cast<int32_t>(prn), chip_shift, c)) return rc;
    return sample_code(c, 1023, 1023000, fs, true, false, dest);
}

extern "C" int gnsship_beidou_b1i_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift)
{
    if (!dest) return GNSSHIP_E_INVAL;
    int8_t c[2046];
    if (int rc = b1i_chips(prn, chip_shift, c)) return rc;
    for (int i = 0; i < 2046; i++) dest[i] = static_cast<float>(c[i]);
    return GNSSHIP_OK;
}

extern "C" int gnsship_beidou_b1i_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t fs, uint32_t chip_shift)
{
    if (!dest) return GNSSHIP_E_INVAL;
    int8_t c[2046];
    if (int rc = b1i_chips(static_cast<int32_t>(prn), chip_shift, c)) return rc;
    return sample_code(c, 2046, 2046000, fs, false, true, dest);
}

extern "C" int gnsship_code_samples_per_code(int32_t chip_rate, int32_t code_len, int32_t fs)
{
    if (chip_rate <= 0 || code_len <= 0 || fs <= 0) return GNSSHIP_E_INVAL;
    return static_cast<int32_t>(static_cast<double>(fs) / (static_cast<double>(chip_rate) / static_cast<double>(code_len)));
}
