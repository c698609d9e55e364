// oracle/ref_codes_harness.cc — extern "C" wrappers around the REFERENCE's own code generators
// (gps_sdr_signal_replica.cc, beidou_b1i_signal_replica.cc), compiled from /root/reference by
// oracle/Makefile with -DHAS_STD_SPAN=1 (the reference's own switch, gps_sdr_signal_replica.h:24).
// TEST INFRASTRUCTURE ONLY: pins oracle/gnss_oracle.c's code generators.
#include "gps_sdr_signal_replica.h"
#include "beidou_b1i_signal_replica.h"
#include <complex>
#include <cstdint>
#include <vector>

extern "C" {
void ref_gps_l1_ca_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift)
{
    gps_l1_ca_code_gen_float(std::span<float>(dest, 1023), prn, chip_shift);
}
int ref_gps_l1_ca_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t fs, uint32_t chip_shift)
{
    const auto n = static_cast<int32_t>(static_cast<double>(fs) / (1023000.0 / 1023.0));
    gps_l1_ca_code_gen_complex_sampled(std::span<std::complex<float>>(reinterpret_cast<std::complex<float>*>(dest), n), prn, fs, chip_shift);
    return n;
}
void ref_beidou_b1i_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift)
{
    beidou_b1i_code_gen_float(std::span<float>(dest, 2046), prn, chip_shift);
}
int ref_beidou_b1i_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t fs, uint32_t chip_shift)
{
    const auto n = static_cast<int32_t>(static_cast<double>(fs) / (2046000.0 / 2046.0));
    beidou_b1i_code_gen_complex_sampled(std::span<std::complex<float>>(reinterpret_cast<std::complex<float>*>(dest), n), prn, fs, chip_shift);
    return n;
}
}
