// tests/cpp/mirror_test.cpp — C++ parity test of the header-only mirror classes
// (include/gnsship_cpp.hpp) against the CPU oracle (oracle/gnss_oracle.c, linked in: test code only).
// Structured like the reference's tracking-lib tests
// (src/tests/unit-tests/signal-processing-blocks/tracking/cpu_multicorrelator_real_codes_test.cc:54-160):
// random uniform input, N in {2048, 4096, 8192}, 1..12 concurrent threads each owning a correlator,
// but with the outputs CHECKED (the reference's test only times them).
//   mirror_test corr   — correlator parity (exit 0 on pass)
//   mirror_test acq    — PCPS acquisition peak parity vs a direct-DFT oracle
//   mirror_test gamma  — prints calculate_threshold's gamma_p_inv for the CPU test (no GPU)
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "gnsship_cpp.hpp"

extern "C" {
int orc_gps_l1_ca_code_gen_float(float* dest, int32_t prn, uint32_t chip_shift);
int orc_gps_l1_ca_code_gen_complex_sampled(float* dest, uint32_t prn, int32_t sampling_freq, uint32_t chip_shift);
int orc_multicorrelator_real_codes(float* corr_out, const float* sig_in, const float* local_code, int code_length_chips,
    const float* shifts_chips, int n_correlators, int high_dyn, float rem_carrier_phase_in_rad, float phase_step_rad,
    float phase_rate_step_rad, float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips,
    int signal_length_samples, float* scratch);
void orc_doppler_wipeoff_grid(float* table, int n_bins, int fft_size, int doppler_max, int doppler_step, int doppler_center,
    int doppler_bias, int64_t fs);
}

static int corr_test()
{
    const int sizes[] = {2048, 4096, 8192};
    const int max_threads = 12;
    float code[1023];
    orc_gps_l1_ca_code_gen_float(code, 1, 0);
    int failures = 0;
    for (int n : sizes) {
        for (int nt = 1; nt <= max_threads; nt += 11) {
            std::vector<std::thread> th;
            std::vector<double> worst(nt, 0.0);
            for (int t = 0; t < nt; t++) {
                th.emplace_back([&, t]() {
                    std::mt19937 gen(1000 + 17 * t + n);
                    std::uniform_real_distribution<float> u(-1.0F, 1.0F);
                    std::vector<std::complex<float>> in(n);
                    for (auto& v : in) v = std::complex<float>(u(gen), u(gen));
                    float shifts[3] = {-0.5F, 0.0F, 0.5F};
                    gnsship::Hip_Multicorrelator_Real_Codes mc;
                    mc.set_rotator(GNSSHIP_ROTATOR_GENERIC);  // the oracle's variant
                    mc.init(n, 3);
                    mc.set_local_code_and_taps(1023, code, shifts);
                    std::complex<float> out[3];
                    mc.set_input_output_vectors(out, in.data());
                    for (int it = 0; it < 4; it++) {
                        const float rem_carr = u(gen) * 3.14F, step = 0.01F * u(gen), rem_code = u(gen), code_step = 0.25575F + 0.0001F * u(gen);
                        if (!mc.Carrier_wipeoff_multicorrelator_resampler(rem_carr, step, 0.0F, rem_code, code_step, 0.0F, n)) {
                            worst[t] = 1e9;
                            return;
                        }
                        float ref[6];
                        orc_multicorrelator_real_codes(ref, reinterpret_cast<const float*>(in.data()), code, 1023, shifts, 3, 0, rem_carr, step, 0.0F,
                            rem_code, code_step, 0.0F, n, nullptr);
                        // noise-only input: relative to the accumulation scale ||x||_2
                        double scale = 0.0;
                        for (auto& v : in) scale += std::norm(std::complex<double>(v));
                        scale = std::sqrt(scale);
                        for (int k = 0; k < 3; k++) {
                            const double e = std::abs(std::complex<double>(out[k]) - std::complex<double>(ref[2 * k], ref[2 * k + 1]));
                            const double r = e / std::max(scale, std::abs(std::complex<double>(ref[2 * k], ref[2 * k + 1])));
                            if (r > worst[t]) worst[t] = r;
                        }
                    }
                    mc.free();
                });
            }
            for (auto& x : th) x.join();
            double w = 0;
            for (double v : worst) w = std::max(w, v);
            // the generic rotator in the reference's serial order: bit for bit (worst = 0)
            std::printf("corr N=%d threads=%d worst_rel_err=%.3e %s\n", n, nt, w, w == 0.0 ? "ok" : "FAIL");
            if (!(w == 0.0)) failures++;
        }
    }
    return failures;
}

static int acq_test()
{
    // fs = 2.048 Msps → fft_size 2048; PRN 12 at fD = -777 Hz, delay 1000 samples, 48 dB-Hz
    gnsship::Acq_Conf conf;
    conf.fs_in = 2048000;
    conf.doppler_max = 5000;
    conf.doppler_step = 500.0F;
    conf.pfa = 0.01F;
    gnsship::Pcps_Acquisition_Hip acq(conf);
    const int n = acq.fft_size();
    std::vector<float> code(2 * n);
    orc_gps_l1_ca_code_gen_complex_sampled(code.data(), 12, 2048000, 0);
    acq.set_local_code(reinterpret_cast<const std::complex<float>*>(code.data()));
    acq.init();
    std::mt19937 gen(7);
    std::normal_distribution<double> g(0.0, 1.0);
    std::vector<std::complex<float>> sig(n);
    const double amp = std::sqrt(2 * std::pow(10.0, 4.8) / 2048000.0);
    float chips[1023];
    orc_gps_l1_ca_code_gen_float(chips, 12, 0);
    for (int i = 0; i < n; i++) {
        const double t = i / 2048000.0;
        const long c = static_cast<long>(std::floor((i - 1000) / 2048000.0 * 1023000.0 * (1 - 777.0 / 1575.42e6)));
        const double cv = chips[((c % 1023) + 1023) % 1023];
        sig[i] = std::complex<float>(amp * cv * std::cos(2 * M_PI * -777.0 * t) + g(gen), amp * cv * std::sin(2 * M_PI * -777.0 * t) + g(gen));
    }
    gnsship::Acq_Outcome out;
    if (!acq.acquisition_core(sig.data(), 123456, out)) return 1;
    // direct-DFT oracle of the |IFFT(FFT(x w) conj(FFT(c)))|² grid = circular cross-correlation
    const int nb = 20;
    std::vector<float> w(2 * static_cast<size_t>(nb) * n);
    orc_doppler_wipeoff_grid(w.data(), nb, n, 5000, 500, 0, 0, 2048000);
    double best = -1;
    int bb = 0, bi = 0;
    for (int b = 0; b < nb; b++) {
        std::vector<std::complex<double>> x(n);
        for (int i = 0; i < n; i++) {
            const std::complex<float> wf(w[2 * (static_cast<size_t>(b) * n + i)], w[2 * (static_cast<size_t>(b) * n + i) + 1]);
            x[i] = std::complex<double>(sig[i] * wf);
        }
        for (int tau = 0; tau < n; tau++) {
            std::complex<double> acc = 0;
            for (int i = 0; i < n; i++) acc += x[(i + tau) % n] * std::complex<double>(code[2 * i], -code[2 * i + 1]);
            const double v = std::norm(acc);
            if (v > best) {
                best = v;
                bb = b;
                bi = tau;
            }
        }
    }
    const double fd = -5000 + 500 * bb;
    std::printf("acq gpu: delay %.1f doppler %.1f stat %.2f thr %.2f positive %d | oracle: delay %d doppler %.1f\n", out.Acq_delay_samples,
        out.Acq_doppler_hz, out.test_statistics, acq.threshold(), out.positive ? 1 : 0, bi, fd);
    return (static_cast<int>(out.Acq_delay_samples) == bi && out.Acq_doppler_hz == fd && out.positive && out.Acq_samplestamp_samples == 123456) ? 0 : 1;
}

// Closed-loop tracking through Dll_Pll_Veml_Tracking_Hip: a synthetic GPS L1 C/A signal (PRN 3,
// 48 dB-Hz, 1500 Hz Doppler) acquired with a 25 Hz / 0.3-sample error; after 300 epochs the
// carrier Doppler must sit within 5 Hz of the truth and every epoch must advance ~4000 samples.
static int trk_test()
{
    const double fs = 4e6, fd = 1500.0, delay_chips = 200.5;
    const double fcode = 1.023e6 * (1.0 + fd / 1575.42e6);
    const int epochs = 300, n = 4000 * (epochs + 3);
    float code[1023];
    orc_gps_l1_ca_code_gen_float(code, 3, 0);
    std::vector<std::complex<float>> x(n);
    std::mt19937 rng(7);
    std::normal_distribution<float> g(0.0F, 1.0F);
    const double amp = std::sqrt(2.0 * std::pow(10.0, 4.8) / fs);
    for (int i = 0; i < n; i++) {
        const double ph = i / fs * fcode - delay_chips;
        const int chip = static_cast<int>(((static_cast<long long>(std::floor(ph)) % 1023) + 1023) % 1023);
        const double car = 2.0 * M_PI * fd * i / fs + 0.3;
        x[i] = std::complex<float>(static_cast<float>(amp * code[chip] * std::cos(car) + g(rng)),
            static_cast<float>(amp * code[chip] * std::sin(car) + g(rng)));
    }
    gnsship::Dll_Pll_Conf conf;
    conf.fs_in = fs;
    conf.vector_length = 4000;
    conf.system = 'G';
    gnsship::Dll_Pll_Veml_Tracking_Hip trk(conf, 2);
    const double delay_samples = delay_chips / fcode * fs + 0.3;
    if (!trk.start_tracking(1, code, nullptr, 1023, delay_samples, fd + 25.0, 0, 0)) {
        std::printf("start_tracking failed: %s\n", trk.last_error());
        return 1;
    }
    std::vector<gnsship_trk_epoch> rec(static_cast<size_t>(epochs) * 2);
    const int done = trk.work(x.data(), 0, n, epochs, rec.data());
    if (done != epochs) {
        std::printf("epochs %d != %d: %s\n", done, epochs, trk.last_error());
        return 1;
    }
    int bad = 0;
    for (int e = 1; e < epochs; e++) {
        const gnsship_trk_epoch& r = rec[static_cast<size_t>(e) * 2 + 1];
        const uint64_t adv = r.sample_counter - rec[static_cast<size_t>(e - 1) * 2 + 1].sample_counter;
        if (!(r.flags & 8) || adv < 3995 || adv > 4005 || rec[static_cast<size_t>(e) * 2].flags) bad++;
    }
    const double dop = rec[static_cast<size_t>(epochs - 1) * 2 + 1].carrier_doppler_hz;
    std::printf("trk: last Doppler %.3f Hz (truth %.1f), state %d, bad epochs %d\n", dop, fd, trk.state(1), bad);
    return (bad == 0 && std::fabs(dop - fd) < 5.0 && trk.state(1) == 2) ? 0 : 1;
}

// Acquisition behind the acquisition resampler: 20.48 Msps IF, Acq_Conf::ConfigureAutomaticResampler(2e6)
// (decimation 10, resampled_fs 2.048 Msps, fft 2048) and Acq_Resampler_Hip in front; PRN 12 at
// fD = 1250 Hz, code start at input sample 10000.  The second 1-ms dwell (warm filter) is acquired.
static int acq_resampler_test()
{
    const int64_t fs = 20480000;
    gnsship::Acq_Conf conf;
    conf.fs_in = fs;
    conf.doppler_max = 5000;
    conf.doppler_step = 250.0F;
    conf.pfa = 0.01F;
    conf.use_automatic_resampler = true;
    conf.ConfigureAutomaticResampler(2000000.0);
    gnsship::Acq_Resampler_Hip rs(fs, 2000000.0, 2 * fs / 1000);
    if (!rs.enabled() || rs.decimation() != 10 || conf.resampler_ratio != 10.0F || conf.resampled_fs != 2048000) {
        std::printf("resampler design mismatch: decimation %d ratio %.1f resampled_fs %lld\n", rs.decimation(), conf.resampler_ratio,
            static_cast<long long>(conf.resampled_fs));
        return 1;
    }
    gnsship::Pcps_Acquisition_Hip acq(conf);
    acq.set_resampler_latency(rs.latency());
    const int n = acq.fft_size();
    std::vector<float> code(2 * n);
    orc_gps_l1_ca_code_gen_complex_sampled(code.data(), 12, 2048000, 0);
    acq.set_local_code(reinterpret_cast<const std::complex<float>*>(code.data()));
    acq.init();
    const int n_in = static_cast<int>(2 * fs / 1000);
    std::mt19937 gen(11);
    std::normal_distribution<double> g(0.0, 1.0);
    std::vector<std::complex<float>> sig(n_in), dec(n_in / 10);
    const double amp = std::sqrt(2 * std::pow(10.0, 4.8) / static_cast<double>(fs));
    float chips[1023];
    orc_gps_l1_ca_code_gen_float(chips, 12, 0);
    for (int i = 0; i < n_in; i++) {
        const double t = i / static_cast<double>(fs);
        const long c = static_cast<long>(std::floor((i - 10000) / static_cast<double>(fs) * 1023000.0 * (1 + 1250.0 / 1575.42e6)));
        const double cv = chips[((c % 1023) + 1023) % 1023];
        sig[i] = std::complex<float>(amp * cv * std::cos(2 * M_PI * 1250.0 * t) + g(gen), amp * cv * std::sin(2 * M_PI * 1250.0 * t) + g(gen));
    }
    if (!rs.work(sig.data(), n_in, dec.data())) return 1;
    gnsship::Acq_Outcome out;
    if (!acq.acquisition_core(dec.data() + n, static_cast<uint64_t>(n), out)) return 1;
    const double period = static_cast<double>(fs) / 1000.0;
    double err = std::fmod(out.Acq_delay_samples - 10000.0 + 1.5 * period, period) - 0.5 * period;
    std::printf("acq resampled: delay %.1f (truth 10000, err %.1f) doppler %.1f stamp %llu stat %.2f thr %.2f positive %d latency %u\n",
        out.Acq_delay_samples, err, out.Acq_doppler_hz, static_cast<unsigned long long>(out.Acq_samplestamp_samples), out.test_statistics,
        acq.threshold(), out.positive ? 1 : 0, rs.latency());
    const bool ok = out.positive && std::fabs(err) <= 20.0 && std::fabs(out.Acq_doppler_hz - 1250.0) <= 250.0 &&
                    out.Acq_samplestamp_samples == static_cast<uint64_t>(10 * n);
    return ok ? 0 : 1;
}

// The block's general_work state machine (pcps_acquisition.cc:902-1031 + decisions :760-864) fed in
// 700-sample pieces: PRN 12 present → ACQ_SUCCESS on the first dwell (samplestamp = one dwell);
// PRN 20 absent with max_dwells = 3 → ACQ_FAIL after three non-coherent dwells.
static int acq_fsm_test()
{
    const int fs = 2048000;
    std::mt19937 gen(5);
    std::normal_distribution<double> g(0.0, 1.0);
    const int total = 20 * fs / 1000;
    std::vector<std::complex<float>> sig(total);
    const double amp = std::sqrt(2 * std::pow(10.0, 4.7) / fs);
    float chips[1023];
    orc_gps_l1_ca_code_gen_float(chips, 12, 0);
    for (int i = 0; i < total; i++) {
        const double t = i / static_cast<double>(fs);
        const long c = static_cast<long>(std::floor((i - 700) / static_cast<double>(fs) * 1023000.0 * (1 + 1500.0 / 1575.42e6)));
        const double cv = chips[((c % 1023) + 1023) % 1023];
        sig[i] = std::complex<float>(amp * cv * std::cos(2 * M_PI * 1500.0 * t) + g(gen), amp * cv * std::sin(2 * M_PI * 1500.0 * t) + g(gen));
    }
    int failures = 0;
    for (int mode = 0; mode < 4; mode++) {  // PRN 12 / 20, blocking / non-blocking worker (:1002-1006)
        const int prn = (mode & 1) ? 20 : 12;
        const bool blocking = mode < 2;
        gnsship::Acq_Conf conf;
        conf.fs_in = fs;
        conf.doppler_max = 5000;
        conf.doppler_step = 500.0F;
        conf.pfa = 0.01F;
        conf.max_dwells = prn == 12 ? 1U : 3U;
        gnsship::Pcps_Acquisition_Hip acq(conf);
        const int n = acq.fft_size();
        std::vector<float> code(2 * n);
        orc_gps_l1_ca_code_gen_complex_sampled(code.data(), prn, fs, 0);
        acq.set_local_code(reinterpret_cast<const std::complex<float>*>(code.data()));
        acq.init();
        acq.blocking = blocking;
        acq.set_state(1);
        int pos = 0, calls = 0;
        gnsship::Pcps_Acquisition_Hip::Acq_Event ev = gnsship::Pcps_Acquisition_Hip::ACQ_NONE;
        while (ev == gnsship::Pcps_Acquisition_Hip::ACQ_NONE && pos < total && calls < 10000) {
            pos += acq.general_work(sig.data() + pos, std::min(700, total - pos), &ev);
            if (!blocking && ev == gnsship::Pcps_Acquisition_Hip::ACQ_NONE) acq.join_worker();  // a GNU Radio scheduler would keep calling
            calls++;
        }
        const auto& r = acq.gnss_synchro();
        std::printf("acq fsm prn %d %s: event %d after %d calls, %d samples; delay %.1f doppler %.1f stamp %llu stat %.2f thr %.2f\n", prn,
            blocking ? "blocking" : "non-blocking",
            static_cast<int>(ev), calls, pos, r.Acq_delay_samples, r.Acq_doppler_hz, static_cast<unsigned long long>(r.Acq_samplestamp_samples),
            r.test_statistics, acq.threshold());
        // non-blocking: the decision is reported by the call after the worker's, which (the block
        // being inactive again) consumes its 700 samples
        const int extra = blocking ? 0 : 700;
        if (prn == 12) {
            const bool ok = ev == gnsship::Pcps_Acquisition_Hip::ACQ_SUCCESS && pos == n + extra && r.Acq_samplestamp_samples == static_cast<uint64_t>(n) &&
                            std::fabs(r.Acq_delay_samples - 700.0) <= 2.0 && std::fabs(r.Acq_doppler_hz - 1500.0) <= 250.0;
            if (!ok) failures++;
        } else {
            const bool ok = ev == gnsship::Pcps_Acquisition_Hip::ACQ_FAIL && pos == 3 * n + extra && r.Acq_samplestamp_samples == static_cast<uint64_t>(3 * n);
            if (!ok) failures++;
        }
    }
    return failures;
}

int main(int argc, char** argv)
{
    const char* mode = argc > 1 ? argv[1] : "corr";
    if (!std::strcmp(mode, "gamma")) {
        const int as[] = {2, 4, 6};
        const double ps[] = {0.5, 0.9, 0.999, 1.0 - 1e-6, 1.0 - 3.125e-8};
        for (int a : as)
            for (double p : ps) std::printf("%d %.17g %.17g\n", a, p, gnsship::gamma_p_inv_int(a, p));
        return 0;
    }
    if (!std::strcmp(mode, "acq")) return acq_test();
    if (!std::strcmp(mode, "acqrs")) return acq_resampler_test();
    if (!std::strcmp(mode, "acqfsm")) return acq_fsm_test();
    if (!std::strcmp(mode, "trk")) return trk_test();
    return corr_test();
}
