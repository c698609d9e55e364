// oracle/ref_trk_harness.cc — extern "C" wrappers around the REFERENCE's own
// Tracking_FLL_PLL_filter (tracking_FLL_PLL_filter.cc) and Exponential_Smoother
// (exponential_smoother.cc), compiled from /root/reference by oracle/Makefile (`ref` target).
// TEST INFRASTRUCTURE ONLY: pins oracle/trk_oracle.c's restatements of those two classes.
#include "exponential_smoother.h"
#include "tracking_FLL_PLL_filter.h"

extern "C" {
// Runs the carrier filter over n (fll, pll, T) triples after set_params + initialize; out[n].
void ref_fll_pll_run(float fll_bw_hz, float pll_bw_hz, int order, float acq_doppler_hz, const float* fll, const float* pll, const float* T,
    int n, float* out)
{
    Tracking_FLL_PLL_filter f;
    f.set_params(fll_bw_hz, pll_bw_hz, order);
    f.initialize(acq_doppler_hz);
    for (int i = 0; i < n; i++) out[i] = f.get_carrier_error(fll[i], pll[i], T[i]);
}
// Exponential_Smoother (float overload) with the setters the tracking block uses.
void ref_smoother_run(float alpha, float min_value, float offset, int samples_for_init, const float* raw, int n, float* out)
{
    Exponential_Smoother s;
    s.set_alpha(alpha);
    s.set_min_value(min_value);
    s.set_offset(offset);
    s.set_samples_for_initialization(samples_for_init);
    for (int i = 0; i < n; i++) out[i] = s.smooth(raw[i]);
}
}
