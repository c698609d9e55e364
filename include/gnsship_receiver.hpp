// gnsship_receiver.hpp — the Channel role over the C ABI: a standalone receiver core that reads an IF
// stream, acquires, hands off to tracking and re-acquires after a loss of lock, the way GNSS-SDR's
// flowgraph drives its channels — without GNU Radio (absent here).
//
// Reference pieces restated (paths relative to the reference root):
//   ChannelFsm                  src/algorithms/channel/libs/channel_fsm.cc:44-220 (states 0 standby,
//                               1 acquisition, 2 tracking, 3 waiting for a satellite; the events)
//   channel_msg_receiver_cc     src/algorithms/channel/libs/channel_msg_receiver_cc.cc:64-100 (acquisition
//                               positive / negative, tracking loss → FSM events; repeat_satellite)
//   Channel                     src/algorithms/channel/adapters/channel.cc:30-108, :215-275 (set_signal →
//                               set_local_code, start_acquisition, assist_acquisition_doppler)
//   GNSSFlowgraph control       src/core/receiver/gnss_flowgraph.cc: set_channels_state :2540-2564,
//                               acquisition_manager :1797-1879, apply_action :1904-2009 (what 0/1/2),
//                               search_next_signal :2615-2629 (GPS 1C), push_back_signal :1652-1660,
//                               remove_signal :1718-1724, set_signals_list :2158-2170 (GPS PRN 1-32)
//   the blocks                  Pcps_Acquisition_Hip::general_work (pcps_acquisition.cc:902-1031) and
//                               Dll_Pll_Veml_Tracking_Hip (dll_pll_veml_tracking.cc) from gnsship_cpp.hpp
//
// Scheduling model (deterministic, one host thread): the stream is processed in blocks.  Within a
// block every channel in acquisition runs its general_work over pieces of `acq_piece` samples (GNU
// Radio's noutput) in stream order; a decision takes effect at the sample where it was made (a positive
// acquisition starts tracking there; a failure hands the next satellite to the next idle channel,
// whose acquisition starts there).  Then the tracking engine runs every tracking channel over the
// block on the device (the closed loop of gnsship_trk_*; each channel continues exactly where it
// stopped, the last 2·vector_length samples of the previous block are kept in front).  A loss of
// lock found in a block re-starts that channel's acquisition at the next block: the control thread's
// reaction latency is one block.  An inactive acquisition consumes the stream as the reference block
// does (its sample counter, hence Acq_samplestamp_samples, is the absolute stream position).
#ifndef GNSSHIP_RECEIVER_HPP
#define GNSSHIP_RECEIVER_HPP

#include <algorithm>
#include <cstdint>
#include <functional>
#include <list>
#include <memory>
#include <string>
#include <vector>

#include "gnsship_cpp.hpp"

namespace gnsship {

// ChannelFsm (channel_fsm.cc:44-220).  The actions are the adapters' calls and the control-queue pushes.
class ChannelFsm {
public:
    std::function<void()> start_acquisition, stop_acquisition, start_tracking, stop_tracking, request_satellite, notify_stop_tracking;
    bool Event_stop_channel()
    {
        if (state_ == 1) {
            state_ = 0;
            stop_acquisition();
        } else if (state_ == 2) {
            state_ = 0;
            stop_tracking();
        }
        return true;
    }
    bool Event_start_acquisition()
    {
        if (state_ == 1 || state_ == 2) return false;
        state_ = 1;
        start_acquisition();
        return true;
    }
    bool Event_valid_acquisition()
    {
        if (state_ != 1) return false;
        state_ = 2;
        start_tracking();
        return true;
    }
    bool Event_failed_acquisition_repeat()
    {
        if (state_ != 1) return false;
        state_ = 1;
        start_acquisition();
        return true;
    }
    bool Event_failed_acquisition_no_repeat()
    {
        if (state_ != 1) return false;
        state_ = 3;
        request_satellite();
        return true;
    }
    bool Event_failed_tracking_standby()
    {
        if (state_ != 2) return false;
        state_ = 0;
        notify_stop_tracking();
        return true;
    }
    unsigned state() const { return state_; }

private:
    unsigned state_ = 0;
};

// The configuration keys of the 1C channels (conf/gnss-sdr_GPS_L1_gr_complex.conf).
struct Receiver_Conf {
    int channels{1};                     // Channels_1C.count
    int in_acquisition{1};               // Channels.in_acquisition (capped at channels)
    std::vector<uint32_t> satellite;     // Channel<i>.satellite (0 or missing: from the search list)
    bool repeat_satellite{false};        // Acquisition_1C.repeat_satellite
    Acq_Conf acq;                        // Acquisition_1C.* (pfa > 0: threshold from calculate_threshold)
    float threshold{0.0F};               // Acquisition_1C.threshold (used when pfa = 0)
    Dll_Pll_Conf trk;                    // Tracking_1C.* (vector_length = round(fs / 1000))
    int64_t block_samples{0};            // processing block (0: 100 ms of samples)
    int acq_piece{8192};                 // samples per acquisition general_work call
    std::string dump_filename;           // Tracking_1C.dump_filename ("" = dump off)
    int device{0};
};

// One control event, in stream order.
struct Receiver_Event {
    uint64_t sample;   // stream position where it took effect
    int channel;
    int what;          // 0 acquisition failed, 1 acquisition positive, 2 tracking lost, 3 acquisition started
    uint32_t prn;
    double doppler_hz, delay_samples;  // acquisition outcome (what 0/1)
    float test_statistic;
};

// One tracking epoch of a channel with the satellite it was tracking (Gnss_Synchro::PRN).
struct Receiver_Record {
    uint32_t prn;
    gnsship_trk_epoch e;
};

class Gnss_Receiver_Hip {
public:
    explicit Gnss_Receiver_Hip(const Receiver_Conf& conf) : conf_(conf), dev_(Device::get(conf.device))
    {
        n_ = std::max(1, conf_.channels);
        max_acq_ = std::min(std::max(0, conf_.in_acquisition), n_);
        conf_.satellite.resize(static_cast<size_t>(n_), 0U);
        if (conf_.trk.vector_length == 0) conf_.trk.vector_length = static_cast<uint32_t>(std::lround(conf_.trk.fs_in / 1000.0));
        vl_ = static_cast<int64_t>(conf_.trk.vector_length);
        block_ = conf_.block_samples > 0 ? conf_.block_samples : static_cast<int64_t>(conf_.trk.fs_in / 10.0);
        tail_ = 2 * vl_;
        trk_ = std::make_unique<Dll_Pll_Veml_Tracking_Hip>(conf_.trk, n_, conf_.device);
        for (uint32_t p = 1; p <= 32; p++) available_.push_back(p);  // set_signals_list (GPS 1C)
        prn_.assign(static_cast<size_t>(n_), 0U);
        apos_.assign(static_cast<size_t>(n_), 0U);
        fsm_.resize(static_cast<size_t>(n_));
        for (int c = 0; c < n_; c++) {
            auto a = std::make_unique<Pcps_Acquisition_Hip>(conf_.acq, conf_.device);
            if (conf_.acq.pfa <= 0.0F) a->set_threshold(conf_.threshold);
            a->set_doppler_step(static_cast<uint32_t>(conf_.acq.doppler_step));
            if (!a->init()) throw std::runtime_error("Pcps_Acquisition_Hip::init failed");
            acq_.push_back(std::move(a));
            wire(c);
        }
        // flowgraph start: satellites assigned in channel order, the first in_acquisition channels acquire
        for (int c = 0; c < n_; c++) set_signal(c, conf_.satellite[static_cast<size_t>(c)] ? conf_.satellite[static_cast<size_t>(c)] : search_next_signal());
        state_.assign(static_cast<size_t>(n_), 0);
        for (int c = 0; c < max_acq_; c++) state_[static_cast<size_t>(c)] = 1;
        acq_count_ = max_acq_;
        for (int c = 0; c < n_; c++)
            if (state_[static_cast<size_t>(c)] == 1) start_acquisition(c);
        drain();
    }

    // Feed the next n samples of the stream (gr_complex).  Returns false on an engine error.
    bool work(const std::complex<float>* x, int64_t n)
    {
        while (n > 0) {
            const int64_t m = std::min(n, block_);
            if (!process_block(x, m)) return false;
            x += m;
            n -= m;
        }
        return true;
    }

    const std::vector<Receiver_Event>& events() const { return events_; }
    // Every tracking epoch record in stream order per channel (the Gnss_Synchro stream).
    const std::vector<std::vector<Receiver_Record>>& records() const { return recs_; }
    uint64_t position() const { return pos_; }
    unsigned channel_fsm_state(int c) const { return fsm_[static_cast<size_t>(c)].state(); }
    uint32_t channel_prn(int c) const { return prn_[static_cast<size_t>(c)]; }
    int tracking_state(int c) { return trk_->state(c); }

private:
    void wire(int c)
    {
        ChannelFsm& f = fsm_[static_cast<size_t>(c)];
        f.start_acquisition = [this, c]() {  // ChannelFsm::start_acquisition → acq_->reset() (set_active)
            skip_idle(c, now_);
            acq_[static_cast<size_t>(c)]->set_active(true);
            apos_[static_cast<size_t>(c)] = now_;
            events_.push_back({now_, c, 3, prn_[static_cast<size_t>(c)], 0.0, 0.0, 0.0F});
        };
        f.stop_acquisition = [this, c]() { acq_[static_cast<size_t>(c)]->set_active(false); };
        f.start_tracking = [this, c]() {  // trk_->start_tracking(); queue (channel, 1)
            const Acq_Outcome& s = acq_[static_cast<size_t>(c)]->gnss_synchro();
            float code[1023];
            gnsship_gps_l1_ca_code_gen_float(code, static_cast<int32_t>(prn_[static_cast<size_t>(c)]), 0);
            if (!trk_->start_tracking(c, code, nullptr, 1023, s.Acq_delay_samples, s.Acq_doppler_hz, s.Acq_samplestamp_samples, now_,
                    static_cast<int>(prn_[static_cast<size_t>(c)])))
                error_ = true;
            queue_.push_back({c, 1});
        };
        f.stop_tracking = [this, c]() { trk_->stop_tracking(c); };
        f.request_satellite = [this, c]() { queue_.push_back({c, 0}); };
        f.notify_stop_tracking = [this, c]() { queue_.push_back({c, 2}); };
    }

    // Channel::set_signal (channel.cc:215-232): new satellite, acq_->set_local_code()
    void set_signal(int c, uint32_t prn)
    {
        prn_[static_cast<size_t>(c)] = prn;
        std::vector<float> code(2 * static_cast<size_t>(acq_[static_cast<size_t>(c)]->consumed_samples()));
        gnsship_gps_l1_ca_code_gen_complex_sampled(code.data(), prn, static_cast<int32_t>(conf_.acq.fs_in), 0);
        if (!acq_[static_cast<size_t>(c)]->set_local_code(reinterpret_cast<const std::complex<float>*>(code.data()))) error_ = true;
    }
    void start_acquisition(int c) { fsm_[static_cast<size_t>(c)].Event_start_acquisition(); }  // Channel::start_acquisition

    // search_next_signal for GPS 1C (gnss_flowgraph.cc:2615-2629): front, rotated to the back
    uint32_t search_next_signal()
    {
        const uint32_t p = available_.front();
        available_.pop_front();
        available_.push_back(p);
        return p;
    }
    void push_back_signal(uint32_t p)
    {
        available_.remove(p);
        available_.push_back(p);
    }

    // acquisition_manager (:1797-1879)
    void acquisition_manager(int who)
    {
        for (int i = 0; i < n_; i++) {
            const int cc = (i + who + 1) % n_;
            if (acq_count_ < max_acq_ && state_[static_cast<size_t>(cc)] == 0) {
                const uint32_t sat = conf_.satellite[static_cast<size_t>(cc)];
                set_signal(cc, sat ? prn_[static_cast<size_t>(cc)] : search_next_signal());
                state_[static_cast<size_t>(cc)] = 1;
                acq_count_++;
                acq_[static_cast<size_t>(cc)]->set_doppler_center(0);  // assist_acquisition_doppler(0)
                start_acquisition(cc);
            }
        }
    }

    // apply_action (:1904-2009) for the channel events
    void apply_action(int who, int what)
    {
        const uint32_t sat = conf_.satellite[static_cast<size_t>(who)];
        const uint32_t gs = prn_[static_cast<size_t>(who)];
        if (what == 0) {
            state_[static_cast<size_t>(who)] = 0;
            if (acq_count_ > 0) acq_count_--;
            acquisition_manager(who);
            if (sat == 0) push_back_signal(gs);
        } else if (what == 1) {
            available_.remove(gs);
            state_[static_cast<size_t>(who)] = 2;
            if (acq_count_ > 0) acq_count_--;
            acquisition_manager(who);
        } else if (what == 2) {
            if (acq_count_ < max_acq_) {
                state_[static_cast<size_t>(who)] = 1;
                acq_count_++;
                set_signal(who, gs);
                start_acquisition(who);
            } else {
                state_[static_cast<size_t>(who)] = 0;
                if (sat == 0) push_back_signal(gs);
            }
        }
    }

    void drain()
    {
        while (!queue_.empty()) {
            const auto ev = queue_.front();
            queue_.erase(queue_.begin());
            apply_action(ev.first, ev.second);
        }
    }

    // an inactive acquisition block consumes the stream (general_work :912-932)
    void skip_idle(int c, uint64_t to)
    {
        Pcps_Acquisition_Hip& a = *acq_[static_cast<size_t>(c)];
        Pcps_Acquisition_Hip::Acq_Event ev;
        a.set_active(false);
        while (a.sample_counter() < to) {
            const int64_t k = std::min<int64_t>(static_cast<int64_t>(to - a.sample_counter()), 1 << 30);
            a.general_work(nullptr, static_cast<int>(k), &ev);
        }
    }

    bool process_block(const std::complex<float>* x, int64_t n)
    {
        const uint64_t b0 = pos_, b1 = pos_ + static_cast<uint64_t>(n);
        // 1. acquisition, in stream order over the channels acquiring
        for (;;) {
            int c = -1;
            for (int i = 0; i < n_; i++)
                if (fsm_[static_cast<size_t>(i)].state() == 1 && apos_[static_cast<size_t>(i)] < b1 &&
                    (c < 0 || apos_[static_cast<size_t>(i)] < apos_[static_cast<size_t>(c)]))
                    c = i;
            if (c < 0) break;
            Pcps_Acquisition_Hip& a = *acq_[static_cast<size_t>(c)];
            const uint64_t p = apos_[static_cast<size_t>(c)];
            const int m = static_cast<int>(std::min<uint64_t>(static_cast<uint64_t>(conf_.acq_piece), b1 - p));
            Pcps_Acquisition_Hip::Acq_Event ev = Pcps_Acquisition_Hip::ACQ_NONE;
            const int used = a.general_work(x + (p - b0), m, &ev);
            apos_[static_cast<size_t>(c)] = p + static_cast<uint64_t>(used);
            now_ = apos_[static_cast<size_t>(c)];
            if (ev != Pcps_Acquisition_Hip::ACQ_NONE) {
                const Acq_Outcome& s = a.gnss_synchro();
                events_.push_back({now_, c, ev == Pcps_Acquisition_Hip::ACQ_SUCCESS ? 1 : 0, prn_[static_cast<size_t>(c)], s.Acq_doppler_hz,
                    s.Acq_delay_samples, s.test_statistics});
                // channel_msg_receiver_cc::msg_handler_channel_events (:64-100)
                ChannelFsm& f = fsm_[static_cast<size_t>(c)];
                if (ev == Pcps_Acquisition_Hip::ACQ_SUCCESS)
                    f.Event_valid_acquisition();
                else if (conf_.repeat_satellite)
                    f.Event_failed_acquisition_repeat();
                else
                    f.Event_failed_acquisition_no_repeat();
                drain();
            } else if (used == 0 && !a.worker_active()) {
                // a decision is pending in state 2 (blocking: the next call makes it); a block that can
                // consume nothing more in this piece ends the channel's turn
                Pcps_Acquisition_Hip::Acq_Event ev2 = Pcps_Acquisition_Hip::ACQ_NONE;
                const int used2 = a.general_work(x + (p - b0), m, &ev2);
                if (used2 == 0 && ev2 == Pcps_Acquisition_Hip::ACQ_NONE) apos_[static_cast<size_t>(c)] = b1;
                else if (ev2 != Pcps_Acquisition_Hip::ACQ_NONE) {
                    apos_[static_cast<size_t>(c)] = p + static_cast<uint64_t>(used2);
                    now_ = apos_[static_cast<size_t>(c)];
                    const Acq_Outcome& s = a.gnss_synchro();
                    events_.push_back({now_, c, ev2 == Pcps_Acquisition_Hip::ACQ_SUCCESS ? 1 : 0, prn_[static_cast<size_t>(c)], s.Acq_doppler_hz,
                        s.Acq_delay_samples, s.test_statistics});
                    ChannelFsm& f = fsm_[static_cast<size_t>(c)];
                    if (ev2 == Pcps_Acquisition_Hip::ACQ_SUCCESS)
                        f.Event_valid_acquisition();
                    else if (conf_.repeat_satellite)
                        f.Event_failed_acquisition_repeat();
                    else
                        f.Event_failed_acquisition_no_repeat();
                    drain();
                } else {
                    apos_[static_cast<size_t>(c)] = p + static_cast<uint64_t>(used2);
                }
            }
            if (error_) return false;
        }
        // 2. tracking over [b0 − tail, b1) on the device
        const size_t keep = static_cast<size_t>(std::min<uint64_t>(static_cast<uint64_t>(tail_), b0 - win_first_));
        if (win_.size() > keep) win_.erase(win_.begin(), win_.end() - static_cast<std::ptrdiff_t>(keep));
        win_first_ = b0 - keep;
        win_.insert(win_.end(), x, x + n);
        const int64_t wn = static_cast<int64_t>(win_.size());
        if (!ensure_dev(static_cast<size_t>(wn) * sizeof(std::complex<float>))) return false;
        {
            std::lock_guard<std::mutex> lk(dev_->mutex());
            if (gnsship_dev_upload(dev_->ctx(), dev_buf_, win_.data(), static_cast<size_t>(wn) * sizeof(std::complex<float>)) != GNSSHIP_OK) return false;
        }
        const int max_ep = static_cast<int>(wn / std::max<int64_t>(1, vl_ - 1)) + 2;
        rec_buf_.assign(static_cast<size_t>(max_ep) * n_, gnsship_trk_epoch{});
        const bool dump = !conf_.dump_filename.empty();
        if (dump) dump_buf_.assign(static_cast<size_t>(max_ep) * n_, gnsship_trk_dump_record{});
        const int rounds = trk_->work_dump(reinterpret_cast<const std::complex<float>*>(dev_buf_), win_first_, wn, max_ep, rec_buf_.data(),
            dump ? dump_buf_.data() : nullptr, true);
        if (rounds < 0) return false;
        recs_.resize(static_cast<size_t>(n_));
        for (int c = 0; c < n_; c++) {
            bool lost = false;
            for (int r = 0; r < rounds; r++) {
                const gnsship_trk_epoch& e = rec_buf_[static_cast<size_t>(r) * n_ + c];
                if (!(e.flags & 8)) continue;  // no epoch of this channel in this round
                recs_[static_cast<size_t>(c)].push_back({prn_[static_cast<size_t>(c)], e});
                if (e.flags & 2) lost = true;
            }
            if (dump) trk_->append_dump_file(conf_.dump_filename, c, rec_buf_.data(), dump_buf_.data(), rounds);
            if (lost) {
                now_ = b1;  // the control thread reacts after the block
                events_.push_back({now_, c, 2, prn_[static_cast<size_t>(c)], 0.0, 0.0, 0.0F});
                fsm_[static_cast<size_t>(c)].Event_failed_tracking_standby();
                drain();
            }
        }
        pos_ = b1;
        now_ = b1;
        return !error_;
    }

    bool ensure_dev(size_t bytes)
    {
        if (bytes <= dev_cap_) return true;
        std::lock_guard<std::mutex> lk(dev_->mutex());
        if (dev_buf_) gnsship_dev_free(dev_->ctx(), dev_buf_);
        dev_buf_ = nullptr;
        dev_cap_ = 0;
        if (gnsship_dev_alloc(dev_->ctx(), bytes, &dev_buf_) != GNSSHIP_OK) return false;
        dev_cap_ = bytes;
        return true;
    }

public:
    ~Gnss_Receiver_Hip()
    {
        if (dev_buf_) gnsship_dev_free(dev_->ctx(), dev_buf_);
    }

private:
    Receiver_Conf conf_;
    std::shared_ptr<Device> dev_;
    int n_ = 1, max_acq_ = 1, acq_count_ = 0;
    int64_t vl_ = 0, block_ = 0, tail_ = 0;
    std::unique_ptr<Dll_Pll_Veml_Tracking_Hip> trk_;
    std::vector<std::unique_ptr<Pcps_Acquisition_Hip>> acq_;
    std::vector<ChannelFsm> fsm_;
    std::vector<uint32_t> prn_;
    std::vector<uint64_t> apos_;
    std::vector<int> state_;  // the flowgraph's channels_state_
    std::list<uint32_t> available_;
    std::vector<std::pair<int, int>> queue_;
    std::vector<Receiver_Event> events_;
    std::vector<std::vector<Receiver_Record>> recs_;
    std::vector<std::complex<float>> win_;
    uint64_t win_first_ = 0, pos_ = 0, now_ = 0;
    void* dev_buf_ = nullptr;
    size_t dev_cap_ = 0;
    std::vector<gnsship_trk_epoch> rec_buf_;
    std::vector<gnsship_trk_dump_record> dump_buf_;
    bool error_ = false;
};

}  // namespace gnsship

#endif  // GNSSHIP_RECEIVER_HPP
