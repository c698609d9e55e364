// gnsship_rx — standalone receiver core over the C ABI: File_Signal_Source → channels (acquisition →
// tracking, re-acquisition after a loss of lock) → per-channel tracking dumps, the Channel role of
// GNSS-SDR without GNU Radio (include/gnsship_receiver.hpp).  Keys mirror the reference's
// configuration (conf/gnss-sdr_GPS_L1_gr_complex.conf); GPS L1 C/A channels.
//
//   gnsship_rx --file F [--item gr_complex|ishort|ibyte] [--fs 4000000] [--seconds S]
//              [--channels 5] [--in-acquisition 1] [--satellite CH:PRN ...] [--repeat-satellite]
//              [--pfa 0.01] [--doppler-max 10000] [--doppler-step 250]
//              [--pll-bw 40] [--dll-bw 4] [--order 3] [--pull-in-time-s 10] [--rotator auto|generic|avx]
//              [--max-carrier-lock-fail 5000] [--max-code-lock-fail 50] [--cn0-min 25]
//              [--block-ms 100] [--acq-piece 8192] [--dump PREFIX] [--events CSV] [--records BIN]
//
// ishort / ibyte samples are converted to gr_complex without scaling (Ishort_To_Complex /
// Ibyte_To_Complex, item_type_helpers.cc:27-73).  stdout: one JSON summary line.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gnsship_receiver.hpp"

namespace {

[[noreturn]] void usage(const char* why)
{
    std::fprintf(stderr, "gnsship_rx: %s\n", why);
    std::exit(2);
}

}  // namespace

int main(int argc, char** argv)
{
    std::string file, item = "gr_complex", dump, events_csv, records_bin, rotator = "auto";
    double fs = 4e6, seconds = 0.0, block_ms = 100.0;
    gnsship::Receiver_Conf rc;
    rc.channels = 5;
    rc.in_acquisition = 1;
    rc.acq.pfa = 0.01F;
    rc.acq.doppler_max = 10000;
    rc.acq.doppler_step = 250.0F;
    rc.trk.pll_bw_hz = 40.0F;
    rc.trk.dll_bw_hz = 4.0F;
    rc.trk.pll_filter_order = 3;
    std::vector<std::pair<int, unsigned>> sats;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) usage(("missing value for " + a).c_str());
            return argv[++i];
        };
        if (a == "--file") file = val();
        else if (a == "--item") item = val();
        else if (a == "--fs") fs = std::atof(val().c_str());
        else if (a == "--seconds") seconds = std::atof(val().c_str());
        else if (a == "--channels") rc.channels = std::atoi(val().c_str());
        else if (a == "--in-acquisition") rc.in_acquisition = std::atoi(val().c_str());
        else if (a == "--satellite") {
            const std::string v = val();
            const size_t k = v.find(':');
            if (k == std::string::npos) usage("--satellite wants CH:PRN");
            sats.push_back({std::atoi(v.substr(0, k).c_str()), static_cast<unsigned>(std::atoi(v.substr(k + 1).c_str()))});
        } else if (a == "--repeat-satellite") rc.repeat_satellite = true;
        else if (a == "--pfa") rc.acq.pfa = static_cast<float>(std::atof(val().c_str()));
        else if (a == "--threshold") rc.threshold = static_cast<float>(std::atof(val().c_str()));
        else if (a == "--doppler-max") rc.acq.doppler_max = std::atoi(val().c_str());
        else if (a == "--doppler-step") rc.acq.doppler_step = static_cast<float>(std::atof(val().c_str()));
        else if (a == "--pll-bw") rc.trk.pll_bw_hz = static_cast<float>(std::atof(val().c_str()));
        else if (a == "--dll-bw") rc.trk.dll_bw_hz = static_cast<float>(std::atof(val().c_str()));
        else if (a == "--order") rc.trk.pll_filter_order = std::atoi(val().c_str());
        else if (a == "--pull-in-time-s") rc.trk.pull_in_time_s = static_cast<uint32_t>(std::atoi(val().c_str()));
        else if (a == "--max-carrier-lock-fail") rc.trk.max_carrier_lock_fail = std::atoi(val().c_str());  // gflags (gnss_sdr_flags.cc)
        else if (a == "--max-code-lock-fail") rc.trk.max_code_lock_fail = std::atoi(val().c_str());
        else if (a == "--cn0-min") rc.trk.cn0_min = std::atoi(val().c_str());
        else if (a == "--rotator") rotator = val();
        else if (a == "--block-ms") block_ms = std::atof(val().c_str());
        else if (a == "--acq-piece") rc.acq_piece = std::atoi(val().c_str());
        else if (a == "--dump") dump = val();
        else if (a == "--events") events_csv = val();
        else if (a == "--records") records_bin = val();
        else usage(("unknown option " + a).c_str());
    }
    if (file.empty()) usage("--file is required");
    const int sample_bytes = item == "gr_complex" ? 8 : item == "ishort" ? 4 : item == "ibyte" ? 2 : 0;
    if (!sample_bytes) usage("--item must be gr_complex, ishort or ibyte");
    rc.acq.fs_in = static_cast<int64_t>(fs);
    rc.trk.fs_in = fs;
    rc.trk.vector_length = static_cast<uint32_t>(std::lround(fs / 1000.0));  // gps_l1_ca_dll_pll_tracking.cc:47
    rc.trk.rotator = rotator == "generic" ? GNSSHIP_ROTATOR_GENERIC : rotator == "avx" ? GNSSHIP_ROTATOR_AVX : GNSSHIP_ROTATOR_AUTO;
    rc.block_samples = static_cast<int64_t>(fs * block_ms / 1000.0);
    rc.dump_filename = dump;
    rc.satellite.assign(static_cast<size_t>(rc.channels), 0U);
    for (const auto& s : sats)
        if (s.first >= 0 && s.first < rc.channels) rc.satellite[static_cast<size_t>(s.first)] = s.second;

    std::FILE* f = std::fopen(file.c_str(), "rb");
    if (!f) usage(("cannot open " + file).c_str());
    if (!dump.empty())
        for (int c = 0; c < rc.channels; c++) std::remove((dump + std::to_string(c) + ".dat").c_str());

    const auto t_init = std::chrono::steady_clock::now();
    gnsship::Gnss_Receiver_Hip rx(rc);
    const int64_t block = rc.block_samples > 0 ? rc.block_samples : static_cast<int64_t>(fs / 10);
    const int64_t limit = seconds > 0 ? static_cast<int64_t>(seconds * fs) : INT64_MAX;
    std::vector<char> raw(static_cast<size_t>(block) * sample_bytes);
    std::vector<std::complex<float>> x(static_cast<size_t>(block));
    int64_t total = 0;
    double io_s = 0.0;
    const auto t0 = std::chrono::steady_clock::now();
    while (total < limit) {
        const auto r0 = std::chrono::steady_clock::now();
        const int64_t want = std::min<int64_t>(block, limit - total);
        const size_t got = std::fread(raw.data(), static_cast<size_t>(sample_bytes), static_cast<size_t>(want), f);
        if (got == 0) break;
        if (item == "gr_complex") {
            std::memcpy(x.data(), raw.data(), got * 8);
        } else if (item == "ishort") {
            const int16_t* s = reinterpret_cast<const int16_t*>(raw.data());
            for (size_t i = 0; i < got; i++) x[i] = {static_cast<float>(s[2 * i]), static_cast<float>(s[2 * i + 1])};
        } else {
            const int8_t* s = reinterpret_cast<const int8_t*>(raw.data());
            for (size_t i = 0; i < got; i++) x[i] = {static_cast<float>(s[2 * i]), static_cast<float>(s[2 * i + 1])};
        }
        io_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - r0).count();
        if (!rx.work(x.data(), static_cast<int64_t>(got))) {
            std::fprintf(stderr, "gnsship_rx: engine error\n");
            return 1;
        }
        total += static_cast<int64_t>(got);
    }
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double init_s = std::chrono::duration<double>(t0 - t_init).count();
    std::fclose(f);

    if (!events_csv.empty()) {
        std::FILE* e = std::fopen(events_csv.c_str(), "w");
        if (e) {
            std::fprintf(e, "sample,channel,what,prn,doppler_hz,delay_samples,test_statistic\n");
            for (const auto& ev : rx.events())
                std::fprintf(e, "%llu,%d,%d,%u,%.17g,%.17g,%.9g\n", static_cast<unsigned long long>(ev.sample), ev.channel, ev.what, ev.prn, ev.doppler_hz,
                    ev.delay_samples, static_cast<double>(ev.test_statistic));
            std::fclose(e);
        }
    }
    if (!records_bin.empty()) {  // per record: int32 channel, int32 prn, then the gnsship_trk_epoch
        std::FILE* r = std::fopen(records_bin.c_str(), "wb");
        if (r) {
            for (int c = 0; c < rc.channels; c++)
                if (c < static_cast<int>(rx.records().size()))
                    for (const auto& e : rx.records()[static_cast<size_t>(c)]) {
                        const int32_t hdr[2] = {c, static_cast<int32_t>(e.prn)};
                        std::fwrite(hdr, sizeof(hdr), 1, r);
                        std::fwrite(&e.e, sizeof(e.e), 1, r);
                    }
            std::fclose(r);
        }
    }
    int n_pos = 0, n_neg = 0, n_lost = 0;
    for (const auto& ev : rx.events()) {
        n_pos += ev.what == 1;
        n_neg += ev.what == 0;
        n_lost += ev.what == 2;
    }
    std::printf("{\"samples\": %lld, \"signal_s\": %.6f, \"wall_s\": %.6f, \"init_s\": %.6f, \"io_s\": %.6f, \"realtime_factor\": %.3f, "
                "\"acq_positive\": %d, \"acq_negative\": %d, \"losses\": %d, \"channels\": [",
        static_cast<long long>(total), static_cast<double>(total) / fs, wall, init_s, io_s, (static_cast<double>(total) / fs) / wall, n_pos, n_neg,
        n_lost);
    for (int c = 0; c < rc.channels; c++) {
        const size_t nr = c < static_cast<int>(rx.records().size()) ? rx.records()[static_cast<size_t>(c)].size() : 0;
        std::printf("%s{\"channel\": %d, \"prn\": %u, \"fsm_state\": %u, \"tracking_state\": %d, \"epochs\": %zu}", c ? ", " : "", c, rx.channel_prn(c),
            rx.channel_fsm_state(c), rx.tracking_state(c), nr);
    }
    std::printf("]}\n");
    return 0;
}
