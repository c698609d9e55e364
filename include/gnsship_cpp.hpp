// gnsship_cpp.hpp — header-only C++ mirror of the reference's engine classes, on top of the C ABI
// (include/gnsship.h).  A GNSS-SDR adapter swaps
//   Cpu_Multicorrelator_Real_Codes  → gnsship::Hip_Multicorrelator_Real_Codes
//   pcps_acquisition's FFT core     → gnsship::Pcps_Acquisition_Hip
// keeping method names, argument meaning and the reference's error behaviour (bool returns;
// configuration errors throw std::invalid_argument like Acq_Conf::SetFromConfiguration,
// acq_conf.cc:28-31).  Only the C ABI crosses the shared-library boundary.
#ifndef GNSSHIP_CPP_HPP
#define GNSSHIP_CPP_HPP

#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "gnsship.h"

namespace gnsship {

// One context (device + stream + code bank) per device, shared by every channel of a process.
class Device {
public:
    static std::shared_ptr<Device> get(int device = 0)
    {
        static std::mutex mu;
        static std::map<int, std::weak_ptr<Device>> live;
        std::lock_guard<std::mutex> lk(mu);
        auto sp = live[device].lock();
        if (!sp) {
            sp = std::shared_ptr<Device>(new Device(device));
            live[device] = sp;
        }
        return sp;
    }
    ~Device()
    {
        if (ctx_) gnsship_ctx_destroy(ctx_);
    }
    gnsship_ctx* ctx() const { return ctx_; }
    std::mutex& mutex() { return mu_; }  // serialises calls that share the context stream

private:
    explicit Device(int device)
    {
        // the library must implement the structs this header was compiled against (gnsship.h ABI notes)
        if (gnsship_abi_version() != GNSSHIP_ABI_VERSION)
            throw std::runtime_error("gnsship: libgnsship ABI " + std::to_string(gnsship_abi_version()) + ", header " +
                                     std::to_string(GNSSHIP_ABI_VERSION));
        if (gnsship_ctx_create(device, &ctx_) != GNSSHIP_OK) throw std::runtime_error("gnsship: no HIP device " + std::to_string(device));
    }
    gnsship_ctx* ctx_ = nullptr;
    std::mutex mu_;
};

// Mirror of Cpu_Multicorrelator_Real_Codes (src/algorithms/tracking/libs/cpu_multicorrelator_real_codes.h:37-61).
class Hip_Multicorrelator_Real_Codes {
public:
    explicit Hip_Multicorrelator_Real_Codes(int device = 0) : dev_(Device::get(device)) {}
    ~Hip_Multicorrelator_Real_Codes() { free(); }
    Hip_Multicorrelator_Real_Codes(const Hip_Multicorrelator_Real_Codes&) = delete;
    Hip_Multicorrelator_Real_Codes& operator=(const Hip_Multicorrelator_Real_Codes&) = delete;

    void set_high_dynamics_resampler(bool use_high_dynamics_resampler)
    {
        high_dyn_ = use_high_dynamics_resampler;
        if (h_) gnsship_corr_set_high_dynamics_resampler(h_, high_dyn_ ? 1 : 0);
    }
    // The volk_gnsssdr rotator variant (GNSSHIP_ROTATOR_*); default AUTO: what the reference's
    // dispatcher runs on this host.  Not part of the reference class (volk chooses there).
    bool set_rotator(int variant)
    {
        rotator_ = variant;
        return !h_ || gnsship_corr_set_rotator(h_, rotator_) == GNSSHIP_OK;
    }
    bool init(int max_signal_length_samples, int n_correlators)
    {
        std::lock_guard<std::mutex> lk(dev_->mutex());
        free_locked();
        n_ = n_correlators;
        if (gnsship_corr_create(dev_->ctx(), max_signal_length_samples, n_correlators, &h_) != GNSSHIP_OK) return false;
        gnsship_corr_set_high_dynamics_resampler(h_, high_dyn_ ? 1 : 0);
        if (gnsship_corr_set_rotator(h_, rotator_) != GNSSHIP_OK) {
            free_locked();
            return false;
        }
        return true;
    }
    // The reference borrows the pointers (:53-63); the device engine copies the code at this call.
    bool set_local_code_and_taps(int code_length_chips, const float* local_code_in, float* shifts_chips)
    {
        if (!h_) return false;
        std::lock_guard<std::mutex> lk(dev_->mutex());
        return gnsship_corr_set_local_code_and_taps(h_, code_length_chips, local_code_in, shifts_chips) == GNSSHIP_OK;
    }
    bool set_input_output_vectors(std::complex<float>* corr_out, const std::complex<float>* sig_in)
    {
        out_ = corr_out;
        in_ = sig_in;
        return true;
    }
    bool Carrier_wipeoff_multicorrelator_resampler(float rem_carrier_phase_in_rad, float phase_step_rad, float phase_rate_step_rad,
        float rem_code_phase_chips, float code_phase_step_chips, float code_phase_rate_step_chips, int signal_length_samples)
    {
        if (!h_ || !out_ || !in_) return false;
        std::vector<float> tmp(2 * static_cast<size_t>(n_));
        int rc;
        {
            std::lock_guard<std::mutex> lk(dev_->mutex());
            rc = gnsship_corr_run(h_, in_, GNSSHIP_FMT_CF32, 0, rem_carrier_phase_in_rad, phase_step_rad, phase_rate_step_rad, rem_code_phase_chips,
                code_phase_step_chips, code_phase_rate_step_chips, signal_length_samples, tmp.data());
        }
        if (rc != GNSSHIP_OK) return false;
        for (int t = 0; t < n_; t++) out_[t] = std::complex<float>(tmp[2 * t], tmp[2 * t + 1]);
        return true;
    }
    bool Carrier_wipeoff_multicorrelator_resampler(float rem_carrier_phase_in_rad, float phase_step_rad, float rem_code_phase_chips,
        float code_phase_step_chips, float code_phase_rate_step_chips, int signal_length_samples)
    {
        return Carrier_wipeoff_multicorrelator_resampler(rem_carrier_phase_in_rad, phase_step_rad, 0.0F, rem_code_phase_chips,
            code_phase_step_chips, code_phase_rate_step_chips, signal_length_samples);
    }
    bool free()
    {
        std::lock_guard<std::mutex> lk(dev_->mutex());
        free_locked();
        return true;
    }
    const char* last_error() const { return gnsship_last_error(dev_->ctx()); }

private:
    void free_locked()
    {
        if (h_) gnsship_corr_destroy(h_);
        h_ = nullptr;
    }
    std::shared_ptr<Device> dev_;
    gnsship_corr* h_ = nullptr;
    int rotator_ = GNSSHIP_ROTATOR_AUTO;
    int n_ = 0;
    bool high_dyn_ = false;  // Dll_Pll_Conf::high_dyn default (dll_pll_conf.h:80)
    std::complex<float>* out_ = nullptr;
    const std::complex<float>* in_ = nullptr;
};

// Mirror of the Acq_Conf fields the PCPS core reads (src/algorithms/acquisition/libs/acq_conf.h:33-81)
// with SetDerivedParams (acq_conf.cc:113-118).
struct Acq_Conf {
    int64_t fs_in{4000000LL};
    float doppler_step{250.0};
    float pfa{0.0};
    uint32_t sampled_ms{1U};
    uint32_t ms_per_code{1U};
    uint32_t chips_per_second{1023000U};
    uint32_t max_dwells{1U};
    int32_t doppler_max{5000};
    bool bit_transition_flag{false};
    bool use_CFAR_algorithm_flag{true};
    bool make_2_steps{false};
    float doppler_step2{125.0};
    uint32_t num_doppler_bins_step2{4U};
    float pfa2{0.0};
    // acquisition resampler (GNSS-SDR.use_acquisition_resampler): resampled_fs = fs_in when unused
    bool use_automatic_resampler{false};
    int64_t resampled_fs{0LL};
    float resampler_ratio{1.0};
    uint32_t resampler_latency_samples{0U};
    // derived
    float samples_per_ms{0.0};
    float samples_per_code{0.0};
    uint32_t samples_per_chip{2U};
    void SetDerivedParams()
    {
        if (pfa < 0.0F || pfa > 1.0F) pfa = 0.0F;       // acq_conf.cc:63-67
        if (pfa <= 0.0F) use_CFAR_algorithm_flag = false;  // :75-79
        if (pfa2 <= 0.0F || pfa2 > 1.0F) pfa2 = pfa;
        if (resampled_fs == 0) resampled_fs = fs_in;       // SetFromConfiguration (:41)
        samples_per_ms = static_cast<float>(resampled_fs) * 0.001F;
        samples_per_chip = static_cast<unsigned int>(std::ceil(static_cast<float>(resampled_fs) / static_cast<float>(chips_per_second)));
        samples_per_code = samples_per_ms * static_cast<float>(ms_per_code);
    }
    // ConfigureAutomaticResampler (acq_conf.cc:91-107), called by the adapters with the signal's
    // optimum acquisition rate (GPS_L1_CA_OPT_ACQ_FS_SPS = 2e6, ...)
    void ConfigureAutomaticResampler(double opt_freq)
    {
        if (!use_automatic_resampler) return;
        if (static_cast<double>(fs_in) > opt_freq) {
            uint32_t decimation = static_cast<uint32_t>(static_cast<double>(fs_in) / opt_freq);
            while (fs_in % decimation > 0) decimation--;
            resampler_ratio = static_cast<float>(decimation);
            resampled_fs = fs_in / static_cast<int>(resampler_ratio);
        }
        SetDerivedParams();
    }
};

// The acquisition resampler the flowgraph puts in front of a channel's acquisition
// (gnss_flowgraph.cc:1028-1113): decimating low-pass FIR designed for the signal's optimum
// acquisition rate.  Feed it the IF stream; its output is the acquisition's input at resampled_fs;
// latency() is what the flowgraph passes to set_resampler_latency.
class Acq_Resampler_Hip {
public:
    Acq_Resampler_Hip(int64_t fs_in, double opt_acq_fs, int64_t max_in_samples, int device = 0) : dev_(Device::get(device))
    {
        int n = 0;
        if (gnsship_acq_resampler_design(fs_in, opt_acq_fs, &decimation_, nullptr, 0, &n) != GNSSHIP_OK)
            throw std::invalid_argument("gnsship_acq_resampler_design");
        taps_.resize(static_cast<size_t>(n));
        if (n > 0) {
            if (gnsship_acq_resampler_design(fs_in, opt_acq_fs, &decimation_, taps_.data(), n, &n) != GNSSHIP_OK)
                throw std::invalid_argument("gnsship_acq_resampler_design");
            std::lock_guard<std::mutex> lk(dev_->mutex());
            if (gnsship_acq_resampler_create(dev_->ctx(), taps_.data(), n, decimation_, max_in_samples, &h_) != GNSSHIP_OK)
                throw std::invalid_argument(std::string("gnsship_acq_resampler_create: ") + gnsship_last_error(dev_->ctx()));
        }
    }
    ~Acq_Resampler_Hip()
    {
        if (h_) gnsship_acq_resampler_destroy(h_);
    }
    bool enabled() const { return h_ != nullptr; }  // false: "input sampling frequency is too low"
    int decimation() const { return decimation_; }
    uint32_t latency() const { return taps_.empty() ? 0U : static_cast<uint32_t>((taps_.size() - 1) / 2); }
    const std::vector<float>& taps() const { return taps_; }
    // n_in gr_complex samples (a multiple of decimation()) -> n_in / decimation() into out
    bool work(const std::complex<float>* in, int64_t n_in, std::complex<float>* out)
    {
        if (!h_) return false;
        std::lock_guard<std::mutex> lk(dev_->mutex());
        return gnsship_acq_resampler_run(h_, in, GNSSHIP_FMT_CF32, 0, n_in, reinterpret_cast<float*>(out), nullptr, nullptr) == GNSSHIP_OK;
    }

private:
    std::shared_ptr<Device> dev_;
    gnsship_acq_resampler* h_ = nullptr;
    int decimation_ = 1;
    std::vector<float> taps_;
};

// What acquisition_core writes into Gnss_Synchro (gnss_synchro.h:52-55; pcps_acquisition.cc:683-696).
struct Acq_Outcome {
    double Acq_delay_samples{0.0};
    double Acq_doppler_hz{0.0};
    uint64_t Acq_samplestamp_samples{0};
    uint32_t Acq_doppler_step{0};
    float test_statistics{0.0F};
    float input_power{0.0F};
    float peak{0.0F};
    bool positive{false};
};

// Regularised lower incomplete gamma P(a, x) for integer a ≥ 1 and its inverse (Newton), the
// boost::math::gamma_p_inv call of pcps_acquisition::calculate_threshold (pcps_acquisition.cc:884-899).
inline double gamma_p_int(int a, double x)
{
    double term = 1.0, sum = 1.0;
    for (int k = 1; k < a; k++) {
        term *= x / k;
        sum += term;
    }
    return 1.0 - std::exp(-x) * sum;
}
inline double gamma_p_inv_int(int a, double p)
{
    if (p <= 0.0) return 0.0;
    if (p >= 1.0) return INFINITY;
    // Q = 1 - p is tiny for CFAR thresholds; iterate on log Q for accuracy.
    const double logq = std::log1p(-p);
    double x = std::max(1.0, a - logq);
    for (int it = 0; it < 100; it++) {
        double term = 1.0, sum = 1.0;
        for (int k = 1; k < a; k++) {
            term *= x / k;
            sum += term;
        }
        const double lq = -x + std::log(sum);  // log Q(a, x)
        double lterm = 1.0;
        for (int k = 1; k < a; k++) lterm *= x / k;  // x^{a-1}/(a-1)!
        const double dlq = -lterm / sum;  // d log Q / dx
        const double step = (lq - logq) / dlq;
        x -= step;
        if (x <= 0.0) x = 1e-12;
        if (std::fabs(step) < 1e-13 * std::max(1.0, x)) break;
    }
    return x;
}

// Mirror of the engine part of pcps_acquisition (pcps_acquisition.cc): set_local_code, init (Doppler
// grid), set_doppler_*, set_threshold, calculate_threshold, acquisition_core over one buffer.
class Pcps_Acquisition_Hip {
public:
    explicit Pcps_Acquisition_Hip(const Acq_Conf& conf, int device = 0) : conf_(conf), dev_(Device::get(device))
    {
        conf_.SetDerivedParams();
        // d_consumed_samples (:71), d_fft_size (:84-91)
        consumed_ = static_cast<int>(conf_.sampled_ms * conf_.samples_per_ms * (conf_.bit_transition_flag ? 2.0 : 1.0));
        fft_size_ = conf_.sampled_ms == conf_.ms_per_code ? consumed_ : 2 * consumed_;
        gnsship_acq_conf c{};
        c.fs_in = conf_.resampled_fs;  // the wipeoff grid runs at the resampled rate (:237)
        c.fft_size = fft_size_;
        c.consumed_samples = consumed_;
        c.bit_transition_flag = conf_.bit_transition_flag ? 1 : 0;
        c.doppler_max = conf_.doppler_max;
        c.doppler_step = static_cast<int32_t>(conf_.doppler_step);
        c.doppler_center = 0;
        c.max_dwells = static_cast<int32_t>(conf_.max_dwells);
        c.use_cfar = conf_.use_CFAR_algorithm_flag ? 1 : 0;
        c.samples_per_chip = static_cast<int32_t>(conf_.samples_per_chip);
        c.samples_per_code = conf_.samples_per_code;
        c.resampler_ratio = conf_.resampler_ratio;
        c.max_prns = 1;
        std::lock_guard<std::mutex> lk(dev_->mutex());
        if (gnsship_acq_create(dev_->ctx(), &c, &h_) != GNSSHIP_OK)
            throw std::invalid_argument(std::string("gnsship_acq_create: ") + gnsship_last_error(dev_->ctx()));
    }
    ~Pcps_Acquisition_Hip()
    {
        if (worker_.joinable()) worker_.join();
        if (h_) gnsship_acq_destroy(h_);
    }
    int fft_size() const { return fft_size_; }
    void set_threshold(float threshold) { threshold_ = threshold; }
    void set_resampler_latency(uint32_t latency_samples) { resampler_latency_ = latency_samples; }  // :168-172
    void set_doppler_max(uint32_t doppler_max) { conf_.doppler_max = static_cast<int32_t>(doppler_max); }
    void set_doppler_step(uint32_t doppler_step) { doppler_step_ = doppler_step; }
    void set_doppler_center(int32_t doppler_center) { doppler_center_ = doppler_center; }
    int consumed_samples() const { return consumed_; }
    // set_local_code (:175-208): FFT of the zero-padded sampled code + conjugate, on the device
    bool set_local_code(const std::complex<float>* code)
    {
        std::lock_guard<std::mutex> lk(dev_->mutex());
        return gnsship_acq_set_local_code(h_, 0, reinterpret_cast<const float*>(code)) == GNSSHIP_OK;
    }
    // init (:248-292): rebuild the Doppler wipeoff grid for the current max/step/center
    bool init()
    {
        std::lock_guard<std::mutex> lk(dev_->mutex());
        const int step = doppler_step_ ? static_cast<int>(doppler_step_) : static_cast<int>(conf_.doppler_step);
        if (gnsship_acq_set_grid(h_, conf_.doppler_max, step, doppler_center_) != GNSSHIP_OK) return false;
        step_two_ = false;
        calculate_threshold();
        return true;
    }
    // calculate_threshold (:884-899)
    void calculate_threshold()
    {
        const float pfa = step_two_ ? conf_.pfa2 : conf_.pfa;
        if (pfa <= 0.0F) return;
        int nb = 0;
        gnsship_acq_num_bins(h_, &nb);
        const int effective_fft_size = conf_.bit_transition_flag ? fft_size_ / 2 : fft_size_;
        const int num_bins = effective_fft_size * nb;
        threshold_ = static_cast<float>(2.0 * gamma_p_inv_int(2 * (conf_.bit_transition_flag ? 1 : static_cast<int>(conf_.max_dwells)),
                                                  std::pow(1.0 - pfa, 1.0 / static_cast<float>(num_bins))));
    }
    bool step_two() const { return step_two_; }
    float threshold() const { return threshold_; }
    // acquisition_core (:600-871) over consumed_samples() gr_complex samples (one dwell).  With
    // make_2_steps a step-one detection switches to the narrow step-two grid around its Doppler
    // (:771-787) and reports positive only from step two; a step-two miss returns to step one.
    bool acquisition_core(const std::complex<float>* in, uint64_t samp_count, Acq_Outcome& out)
    {
        gnsship_acq_result r{};
        {
            std::lock_guard<std::mutex> lk(dev_->mutex());
            if (gnsship_acq_run(h_, in, GNSSHIP_FMT_CF32, 0, 1, &r, nullptr) != GNSSHIP_OK) return false;
        }
        out.Acq_delay_samples = r.acq_delay_samples - static_cast<double>(resampler_latency_);  // :686-687
        out.Acq_doppler_hz = static_cast<double>(r.doppler_hz);
        out.Acq_samplestamp_samples = static_cast<uint64_t>(std::rint(static_cast<double>(samp_count) * conf_.resampler_ratio));  // :689
        out.Acq_doppler_step = step_two_ ? static_cast<uint32_t>(conf_.doppler_step2) : out.Acq_doppler_step;
        out.test_statistics = r.test_statistic;
        if (!step_two_) last_input_power_ = r.input_power;
        out.input_power = step_two_ ? last_input_power_ : r.input_power;
        out.peak = r.peak;
        const bool hit = r.test_statistic > threshold_;
        out.positive = hit && (!conf_.make_2_steps || step_two_);
        if (conf_.make_2_steps) {
            std::lock_guard<std::mutex> lk(dev_->mutex());
            if (hit && !step_two_) {
                if (gnsship_acq_set_grid_step2(h_, static_cast<float>(r.doppler_hz), conf_.doppler_step2,
                        static_cast<int>(conf_.num_doppler_bins_step2), r.input_power) != GNSSHIP_OK)
                    return false;
                step_two_ = true;
            } else if (step_two_) {
                const int step = doppler_step_ ? static_cast<int>(doppler_step_) : static_cast<int>(conf_.doppler_step);
                if (gnsship_acq_set_grid(h_, conf_.doppler_max, step, doppler_center_) != GNSSHIP_OK) return false;
                step_two_ = false;
            }
        }
        calculate_threshold();
        return true;
    }
    const char* last_error() const { return gnsship_last_error(dev_->ctx()); }

    // ---- the block's buffering / decision state machine (general_work :902-1031, blocking mode,
    // with the decision part of acquisition_core :760-864) ----
    enum Acq_Event { ACQ_NONE = 0, ACQ_SUCCESS = 1, ACQ_FAIL = 2 };  // the channel messages (:339-390)
    // set_active (:344-352 of the header) / set_state (:315-336)
    void set_active(bool active) { active_ = active; }
    void set_state(int state)
    {
        fsm_state_ = state;
        if (state == 1) {
            synchro_ = Acq_Outcome{};
            active_ = true;
        }
    }
    bool blocking_on_standby{false};  // Acq_Conf::blocking_on_standby
    // Acq_Conf::blocking (acq_conf.h, default true).  false: state 2 runs acquisition_core in a worker
    // thread that holds the block's lock while it runs (pcps_acquisition.cc:602,1002-1006); general_work
    // returns at once and, while the worker is active, consumes input only when the last dwell is in
    // flight (:918-932).  The worker's decision is reported by the next general_work call.
    bool blocking{true};
    uint64_t sample_counter() const { return sample_counter_; }
    const Acq_Outcome& gnss_synchro() const { return synchro_; }
    bool worker_active() const { return worker_active_; }
    // One general_work call over n gr_complex samples: returns how many it consumed (consume_each)
    // and, when acquisition_core ran and decided, ACQ_SUCCESS / ACQ_FAIL in *event.
    int general_work(const std::complex<float>* in, int n, Acq_Event* event)
    {
        std::unique_lock<std::mutex> lk(set_lock_);  // d_setlock (:917)
        *event = pending_event_;
        pending_event_ = ACQ_NONE;
        if (!active_ || worker_active_) {
            const bool consume = !active_ || (worker_active_ && counter_ == conf_.max_dwells);
            const int c = (!blocking_on_standby && consume) ? n : 0;
            sample_counter_ += static_cast<uint64_t>(c);
            if (step_two_) {
                fsm_state_ = 0;
                active_ = true;
            }
            return c;
        }
        switch (fsm_state_) {
        case 0: {
            synchro_ = Acq_Outcome{};
            fsm_state_ = 1;
            buffer_count_ = 0;
            if (blocking_on_standby) return 0;
            sample_counter_ += static_cast<uint64_t>(n);
            return n;
        }
        case 1: {
            if (buffer_.size() != static_cast<size_t>(consumed_)) buffer_.assign(static_cast<size_t>(consumed_), std::complex<float>{});
            const int inc = (n + buffer_count_ <= consumed_) ? n : consumed_ - buffer_count_;
            std::copy(in, in + inc, buffer_.begin() + buffer_count_);
            if (buffer_count_ >= consumed_) fsm_state_ = 2;  // checked before the increment, as :967-970
            buffer_count_ += inc;
            sample_counter_ += static_cast<uint64_t>(inc);
            return inc;
        }
        default: {
            if (blocking) {
                decide(buffer_.data(), event);
            } else {
                if (worker_.joinable()) worker_.join();  // the previous worker has released the lock
                worker_active_ = true;
                worker_ = std::thread([this]() {
                    std::lock_guard<std::mutex> g(set_lock_);  // acquisition_core holds d_setlock (:602)
                    Acq_Event ev = ACQ_NONE;
                    decide(buffer_.data(), &ev);
                    worker_active_ = false;  // :858
                    pending_event_ = ev;
                });
            }
            buffer_count_ = 0;
            return 0;
        }
        }
    }
    // Wait for a non-blocking acquisition_core in flight (its decision is then pending for the next
    // general_work call).
    void join_worker()
    {
        if (worker_.joinable()) worker_.join();
    }

private:
    // acquisition_core's counter update, core and decision block (:623, :683-696, :760-864)
    void decide(const std::complex<float>* in, Acq_Event* event)
    {
        counter_++;
        gnsship_acq_result r{};
        {
            std::lock_guard<std::mutex> lk(dev_->mutex());
            if (gnsship_acq_run(h_, in, GNSSHIP_FMT_CF32, 0, 1, &r, nullptr) != GNSSHIP_OK) return;
        }
        synchro_.Acq_delay_samples = r.acq_delay_samples - static_cast<double>(resampler_latency_);
        synchro_.Acq_doppler_hz = static_cast<double>(r.doppler_hz);
        synchro_.Acq_samplestamp_samples = static_cast<uint64_t>(std::rint(static_cast<double>(sample_counter_) * conf_.resampler_ratio));
        synchro_.Acq_doppler_step = step_two_ ? static_cast<uint32_t>(conf_.doppler_step2) : static_cast<uint32_t>(conf_.doppler_step);
        synchro_.test_statistics = r.test_statistic;
        if (!step_two_) last_input_power_ = r.input_power;
        synchro_.input_power = step_two_ ? last_input_power_ : r.input_power;
        synchro_.peak = r.peak;
        bool positive_acq = false;
        const bool hit = r.test_statistic > threshold_;
        auto to_step_one = [&]() {
            const int step = doppler_step_ ? static_cast<int>(doppler_step_) : static_cast<int>(conf_.doppler_step);
            std::lock_guard<std::mutex> lk(dev_->mutex());
            gnsship_acq_set_grid(h_, conf_.doppler_max, step, doppler_center_);
            step_two_ = false;
        };
        auto on_hit = [&]() {
            if (conf_.make_2_steps) {
                if (step_two_) {
                    *event = ACQ_SUCCESS;
                    positive_acq = true;
                    to_step_one();
                    fsm_state_ = 0;
                } else {
                    std::lock_guard<std::mutex> lk(dev_->mutex());
                    gnsship_acq_set_grid_step2(h_, static_cast<float>(r.doppler_hz), conf_.doppler_step2, static_cast<int>(conf_.num_doppler_bins_step2),
                        r.input_power);
                    step_two_ = true;
                    counter_ = 0;
                    fsm_state_ = 0;
                }
                calculate_threshold();
            } else {
                *event = ACQ_SUCCESS;
                positive_acq = true;
                fsm_state_ = 0;
            }
        };
        if (!conf_.bit_transition_flag) {
            if (hit) {
                active_ = false;
                on_hit();
            } else {
                fsm_state_ = 1;
            }
            if (counter_ == conf_.max_dwells) {
                if (fsm_state_ != 0) *event = ACQ_FAIL;
                fsm_state_ = 0;
                active_ = false;
                if (step_two_) {
                    to_step_one();
                    calculate_threshold();
                }
            }
        } else {
            active_ = false;
            if (hit) {
                on_hit();
            } else {
                fsm_state_ = 0;
                if (step_two_) {
                    to_step_one();
                    calculate_threshold();
                }
                *event = ACQ_FAIL;
            }
        }
        if (counter_ == conf_.max_dwells || positive_acq || conf_.bit_transition_flag) counter_ = 0;
        if (counter_ == 0) {
            std::lock_guard<std::mutex> lk(dev_->mutex());
            gnsship_acq_reset_dwells(h_);
        }
    }

    std::mutex set_lock_;
    std::thread worker_;
    bool worker_active_ = false;
    Acq_Event pending_event_ = ACQ_NONE;
    bool active_ = false;
    int fsm_state_ = 0;
    int buffer_count_ = 0;
    uint32_t counter_ = 0;
    uint64_t sample_counter_ = 0;
    std::vector<std::complex<float>> buffer_;
    Acq_Outcome synchro_{};
    Acq_Conf conf_;
    std::shared_ptr<Device> dev_;
    gnsship_acq* h_ = nullptr;
    int fft_size_ = 0;
    int consumed_ = 0;
    bool step_two_ = false;
    float last_input_power_ = 0.0F;
    float threshold_ = 0.0F;
    uint32_t doppler_step_ = 0;
    int32_t doppler_center_ = 0;
    uint32_t resampler_latency_ = 0;
};

// Mirror of Dll_Pll_Conf (src/algorithms/tracking/libs/dll_pll_conf.h:33-80): same field names and
// defaults (FLAGS_* defaults from gnss_sdr_flags.cc:48-57 for the lock-detector fields).
struct Dll_Pll_Conf {
    double fs_in{2000000.0};
    double carrier_lock_th{0.7};
    float pll_bw_hz{35.0F}, dll_bw_hz{2.0F}, fll_bw_hz{35.0F};
    float early_late_space_chips{0.25F}, very_early_late_space_chips{0.5F};
    float early_late_space_narrow_chips{0.15F}, very_early_late_space_narrow_chips{0.5F};
    float pll_bw_narrow_hz{5.0F}, dll_bw_narrow_hz{0.75F};
    int32_t extend_correlation_symbols{1};
    bool enable_fll_pull_in{false}, enable_fll_steady_state{false};
    bool high_dyn{false};
    uint32_t smoother_length{10U};
    float slope{1.0F}, spc{0.5F}, y_intercept{1.0F};
    float cn0_smoother_alpha{0.002F}, carrier_lock_test_smoother_alpha{0.002F};
    uint32_t pull_in_time_s{10U}, bit_synchronization_time_limit_s{20U}, vector_length{0U};
    int32_t pll_filter_order{3}, dll_filter_order{2};
    int32_t cn0_samples{20}, cn0_smoother_samples{200}, carrier_lock_test_smoother_samples{25}, cn0_min{25};
    int32_t max_code_lock_fail{50}, max_carrier_lock_fail{5000};
    bool carrier_aiding{true}, track_pilot{true};
    char system{'G'};    // 'G' GPS L1 C/A, 'E' Galileo E1, 'C' BeiDou B1I
    char signal[3]{"1C"};
    // Not a Dll_Pll_Conf member: the reference's correlations follow the volk_gnsssdr rotator variant
    // its dispatcher picks on the host (volk_gnsssdr_rank_archs.c); AUTO makes the same choice.
    int32_t rotator{GNSSHIP_ROTATOR_AUTO};
    // Not a Dll_Pll_Conf member either: InputFilter<i>.IF of the signal's conditioner (the reference removes
    // it ahead of the channels; here the correlator NCO wipes it off, gnsship.h if_hz).
    double if_hz{0.0};
};

// Mirror of dll_pll_veml_tracking (gnuradio_blocks/dll_pll_veml_tracking.cc) for many channels on one
// device: start_tracking(:643-883) per channel, general_work over an IF buffer for all of them (the
// per-epoch loop runs on the device; one record per channel-epoch).
class Dll_Pll_Veml_Tracking_Hip {
public:
    Dll_Pll_Veml_Tracking_Hip(const Dll_Pll_Conf& conf, int max_channels, int device = 0) : dev_(Device::get(device)), channels_(max_channels)
    {
        gnsship_trk_conf c{};
        c.fs_in = conf.fs_in;
        c.carrier_lock_th = conf.carrier_lock_th;
        c.pll_bw_hz = conf.pll_bw_hz;
        c.dll_bw_hz = conf.dll_bw_hz;
        c.fll_bw_hz = conf.fll_bw_hz;
        c.early_late_space_chips = conf.early_late_space_chips;
        c.very_early_late_space_chips = conf.very_early_late_space_chips;
        c.slope = conf.slope;
        c.spc = conf.spc;
        c.y_intercept = conf.y_intercept;
        c.cn0_smoother_alpha = conf.cn0_smoother_alpha;
        c.carrier_lock_test_smoother_alpha = conf.carrier_lock_test_smoother_alpha;
        c.pull_in_time_s = conf.pull_in_time_s;
        c.bit_synchronization_time_limit_s = conf.bit_synchronization_time_limit_s;
        c.vector_length = conf.vector_length;
        c.pll_filter_order = conf.pll_filter_order;
        c.dll_filter_order = conf.dll_filter_order;
        c.cn0_samples = conf.cn0_samples;
        c.cn0_smoother_samples = conf.cn0_smoother_samples;
        c.carrier_lock_test_smoother_samples = conf.carrier_lock_test_smoother_samples;
        c.cn0_min = conf.cn0_min;
        c.max_code_lock_fail = conf.max_code_lock_fail;
        c.max_carrier_lock_fail = conf.max_carrier_lock_fail;
        c.carrier_aiding = conf.carrier_aiding ? 1 : 0;
        c.track_pilot = conf.track_pilot ? 1 : 0;
        c.extend_correlation_symbols = conf.extend_correlation_symbols;
        c.pll_bw_narrow_hz = conf.pll_bw_narrow_hz;
        c.dll_bw_narrow_hz = conf.dll_bw_narrow_hz;
        c.early_late_space_narrow_chips = conf.early_late_space_narrow_chips;
        c.very_early_late_space_narrow_chips = conf.very_early_late_space_narrow_chips;
        c.enable_fll_pull_in = conf.enable_fll_pull_in ? 1 : 0;
        c.enable_fll_steady_state = conf.enable_fll_steady_state ? 1 : 0;
        c.high_dyn = conf.high_dyn ? 1 : 0;
        c.smoother_length = conf.smoother_length;
        c.rotator = conf.rotator;
        c.if_hz = conf.if_hz;
        c.system = conf.system == 'E' ? GNSSHIP_SYS_GAL_E1 : conf.system == 'C' ? GNSSHIP_SYS_BDS_B1I : GNSSHIP_SYS_GPS_L1CA;
        code_base_ = 1024 + 2 * max_channels * next_engine_id();
        std::lock_guard<std::mutex> lk(dev_->mutex());
        if (gnsship_trk_create(dev_->ctx(), &c, max_channels, &h_) != GNSSHIP_OK)
            throw std::invalid_argument(std::string("gnsship_trk_create: ") + gnsship_last_error(dev_->ctx()));
    }
    ~Dll_Pll_Veml_Tracking_Hip()
    {
        if (h_) gnsship_trk_destroy(h_);
    }
    // start_tracking for one channel: the local code(s) as the block generates them (d_tracking_code,
    // d_data_code; code_len = samples per chip × chips) and the acquisition's Gnss_Synchro fields
    // (prn selects the BeiDou GEO symbol synchronisation).
    bool start_tracking(int channel, const float* tracking_code, const float* data_code, int code_len, double acq_delay_samples,
        double acq_doppler_hz, uint64_t acq_samplestamp_samples, uint64_t first_sample, int prn = 0)
    {
        if (channel < 0 || channel >= channels_) return false;
        std::lock_guard<std::mutex> lk(dev_->mutex());
        const int cid = code_base_ + 2 * channel;
        if (gnsship_code_set(dev_->ctx(), cid, tracking_code, code_len) != GNSSHIP_OK) return false;
        if (data_code && gnsship_code_set(dev_->ctx(), cid + 1, data_code, code_len) != GNSSHIP_OK) return false;
        gnsship_trk_start_args a{};
        a.code_id = cid;
        a.data_code_id = data_code ? cid + 1 : -1;
        a.acq_delay_samples = acq_delay_samples;
        a.acq_doppler_hz = acq_doppler_hz;
        a.acq_samplestamp_samples = acq_samplestamp_samples;
        a.first_sample = first_sample;
        a.prn = prn;
        return gnsship_trk_start(h_, channel, &a) == GNSSHIP_OK;
    }
    bool stop_tracking(int channel)
    {
        std::lock_guard<std::mutex> lk(dev_->mutex());
        return gnsship_trk_stop(h_, channel) == GNSSHIP_OK;
    }
    // msg_handler_telemetry_to_trk (dll_pll_veml_tracking.cc:617-640): the telemetry decoder's
    // fault message (event 1) forces loss of lock at the channel's next lock check
    bool msg_handler_telemetry_to_trk(int channel, int tlm_event)
    {
        std::lock_guard<std::mutex> lk(dev_->mutex());
        return gnsship_trk_telemetry_event(h_, channel, tlm_event) == GNSSHIP_OK;
    }
    // general_work for every channel over gr_complex samples [first_sample, first_sample + n): up to
    // max_epochs epochs per channel; records (max_epochs × max_channels, optional) as gnsship_trk_epoch.
    int work(const std::complex<float>* in, uint64_t first_sample, int64_t n, int max_epochs, gnsship_trk_epoch* records = nullptr,
        bool in_on_device = false)
    {
        int done = 0;
        std::lock_guard<std::mutex> lk(dev_->mutex());
        if (gnsship_trk_run(h_, in, GNSSHIP_FMT_CF32, in_on_device ? 1 : 0, first_sample, n, max_epochs, records, &done) != GNSSHIP_OK) return -1;
        return done;
    }
    // work() with Dll_Pll_Conf::dump on: dumps (max_epochs × max_channels) receives the log_data
    // records (:1376-1466) of the epochs whose record has flags & 16.
    int work_dump(const std::complex<float>* in, uint64_t first_sample, int64_t n, int max_epochs, gnsship_trk_epoch* records,
        gnsship_trk_dump_record* dumps, bool in_on_device = false)
    {
        int done = 0;
        std::lock_guard<std::mutex> lk(dev_->mutex());
        if (gnsship_trk_run_dump(h_, in, GNSSHIP_FMT_CF32, in_on_device ? 1 : 0, first_sample, n, max_epochs, records, dumps, &done) !=
            GNSSHIP_OK)
            return -1;
        return done;
    }
    // Append channel `channel`'s records to its dump file (<dump_filename><channel>.dat, as the
    // block's d_dump_file): the binary layout tracking_dump_reader reads.
    bool append_dump_file(const std::string& dump_filename, int channel, const gnsship_trk_epoch* records, const gnsship_trk_dump_record* dumps,
        int rounds) const
    {
        const std::string path = dump_filename + std::to_string(channel) + ".dat";
        std::FILE* f = std::fopen(path.c_str(), "ab");
        if (!f) return false;
        bool ok = true;
        for (int r = 0; r < rounds && ok; r++) {
            const size_t i = static_cast<size_t>(r) * channels_ + channel;
            if (records[i].flags & 16) ok = std::fwrite(&dumps[i], sizeof(gnsship_trk_dump_record), 1, f) == 1;
        }
        return std::fclose(f) == 0 && ok;
    }
    int state(int channel, uint64_t* next_sample = nullptr)
    {
        int st = -1;
        std::lock_guard<std::mutex> lk(dev_->mutex());
        gnsship_trk_channel_state(h_, channel, &st, next_sample);
        return st;
    }
    const char* last_error() const { return gnsship_last_error(dev_->ctx()); }

private:
    static int next_engine_id()
    {
        static std::atomic<int> n{0};
        return n++;
    }
    std::shared_ptr<Device> dev_;
    gnsship_trk* h_ = nullptr;
    int channels_ = 0;
    int code_base_ = 0;
};

}  // namespace gnsship

#endif  // GNSSHIP_CPP_HPP
