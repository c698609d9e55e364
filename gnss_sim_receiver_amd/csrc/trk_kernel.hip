// trk_kernel.hip — device-resident DLL/PLL tracking loop, one lane per channel.
//
// Per round the host enqueues, without synchronising:
//   trk_step_kernel(consume, emit) → corr_anchor_kernel → corr_batch_kernel(s) → corr_reduce_kernel
// The step kernel consumes the correlations of the epoch that just ran (state machine of
// dll_pll_veml_tracking::general_work states 2 and 4) and writes the next epoch's correlator
// jobs in place (the job/chunk plan is fixed: every epoch correlates vector_length samples,
// :1049), so the same launch sequence repeats with no host round trip.
//
// Reference functions restated here (types as in the reference):
//   Tracking_loop_filter::apply           tracking_loop_filter.cc:58-84
//   Tracking_FLL_PLL_filter::get_carrier_error   tracking_FLL_PLL_filter.cc:72-110
//   pll_cloop_two_quadrant_atan / pll_four_quadrant_atan / dll_nc_e_minus_l_normalized /
//   dll_nc_vemlp_normalized               tracking_discriminators.cc:99-160
//   cn0_m2m4_estimator / carrier_lock_detector   lock_detectors.cc:90-147
//   Exponential_Smoother::smooth(float)   exponential_smoother.cc:76-105
//   cn0_and_tracking_lock_status :972-1029, run_dll_pll :1065-1152, update_tracking_vars
//   :1189-1260, save_correlation_results :1262-1350, acquire_secondary :925-970,
//   general_work states 2 (:1789-1932) and 4 (:1971-2028).
// The job derivation repeats derive_job (gnsship_abi.hip) on the device, the phasors with glibc's
// cosf / sinf restated (glibc_sincosf.h), as the host path calls them.
#include <cmath>

#include "anchor_replay.h"
#include "trk_engine.h"
#include "trk_loop.h"

namespace gnsship {

namespace {

// derive_job (gnsship_abi.hip) for a tracking epoch; the plan fields of `j` are kept.
__device__ void fill_job(DevJob& j, const TrkParams& k, const TrkChannel& c, int64_t offset, int code_id, int n_taps, const float* shifts)
{
    const float spcf = static_cast<float>(k.code_samples_per_chip);
    const float rem_carr = corr_rem_carr(k, c);
    const float step = corr_phase_step(k, c);
    float sr, cr, si, ci;
    glibc_sincosf(rem_carr, &sr, &cr);
    glibc_sincosf(-step, &si, &ci);
    const float p0r = cr, p0i = -sr;
    const float incr = ci, inci = si;
    j.sample_offset = offset;
    j.n_samples = static_cast<int32_t>(k.conf.vector_length);
    j.code_id = code_id;
    j.n_taps = n_taps;
    j.p0_re = p0r;
    j.p0_im = p0i;
    j.inc_re = incr;
    j.inc_im = inci;
    j.dtheta = atan2(static_cast<double>(inci), static_cast<double>(incr));
    j.log_mag_inc = static_cast<float>(log(hypot(static_cast<double>(incr), static_cast<double>(inci))));
    j.rot_avx = 0;
    j.rem_code = __fmul_rn(static_cast<float>(c.rem_code_phase_chips), spcf);
    j.code_step = __fmul_rn(static_cast<float>(c.code_phase_step_chips), spcf);
    j.in_margin = 0;  // the tracking plan launches the general (wrapping) chip-index path
    for (int t = 0; t < kMaxTaps; t++) j.shifts[t] = t < n_taps ? shifts[t] : 0.0f;
}

// derive_hd_job (corr_hd_kernel.hip) for a tracking epoch with the smoothed rates
// (do_correlation_step :1041-1048); the plan fields and the code replica of `j` are kept.
__device__ void fill_hd_job(HdJob& j, const TrkParams& k, const TrkChannel& c, int64_t offset, int n_taps, const float* shifts)
{
    const float spcf = static_cast<float>(k.code_samples_per_chip);
    const float rem_carr = corr_rem_carr(k, c);
    const float step = corr_phase_step(k, c);
    const float rate = static_cast<float>(c.carrier_phase_rate_step_rad);
    j.sample_offset = offset;
    j.n_samples = static_cast<int32_t>(k.conf.vector_length);
    j.n_taps = n_taps;
    float sr, cr, si, ci;
    glibc_sincosf(rem_carr, &sr, &cr);
    glibc_sincosf(-step, &si, &ci);
    j.p0_re = cr;
    j.p0_im = -sr;
    j.inc_re = ci;
    j.inc_im = si;
    j.dtheta = atan2(static_cast<double>(j.inc_im), static_cast<double>(j.inc_re));
    j.log_mag_inc = static_cast<float>(log(hypot(static_cast<double>(j.inc_re), static_cast<double>(j.inc_im))));
    j.rate_arg = atan2f(sinf(-rate), cosf(-rate));
    j.rem_code = __fmul_rn(static_cast<float>(c.rem_code_phase_chips), spcf);
    j.code_step = __fmul_rn(static_cast<float>(c.code_phase_step_chips), spcf);
    j.code_rate = __fmul_rn(static_cast<float>(c.code_phase_rate_step_chips), spcf);
    j.shift0 = shifts[0];
    // cumulative circular shifts (…_high_dynamics_resampler_32f_xn.h:83-90); tracking taps increase,
    // so the sum stays within [0, N] (clamped for safety: a shift of N is the identity)
    uint32_t sum = 0;
    j.shift_samples[0] = 0;
    for (int t = 1; t < kMaxTaps; t++) {
        if (t < n_taps) {
            const float q = __fdiv_rn(__fsub_rn(shifts[t], shifts[t - 1]), j.code_step);
            sum += static_cast<uint32_t>(static_cast<int>(round(static_cast<double>(q))));
            if (sum > static_cast<uint32_t>(j.n_samples)) sum = static_cast<uint32_t>(j.n_samples);
        }
        j.shift_samples[t] = t < n_taps ? sum : 0u;
    }
}

__global__ void trk_step_kernel(const TrkParams* __restrict__ pk, TrkChannel* __restrict__ chans, int n_chans, DevJob* __restrict__ jobs,
    ChunkDesc* __restrict__ chunks, const float* __restrict__ corr_out, uint64_t buf_first, int64_t buf_len, int consume, int emit,
    gnsship_trk_epoch* __restrict__ rec, gnsship_trk_dump_record* __restrict__ dump, int* __restrict__ ran_count, TrkHist* __restrict__ hist,
    HdJob* __restrict__ hd_jobs, HdChunk* __restrict__ hd_chunks, Anchor* __restrict__ anchors)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_chans) return;
    const TrkParams& k = *pk;
    TrkChannel c = chans[i];
    const int jb = i * k.jobs_per_channel;
    if (consume && c.ran) {
        gnsship_trk_epoch r = {};
        r.flags = 8;
        const float* taps = corr_out + static_cast<int64_t>(jb) * 2 * kMaxTaps;
        const float* pdata = k.jobs_per_channel > 1 ? corr_out + static_cast<int64_t>(jb + 1) * 2 * kMaxTaps : taps;
        gnsship_trk_dump_record dr;
        epoch_update(k, c, taps, pdata, r, hist ? hist + i : nullptr, dump ? &dr : nullptr);
        if (dump && (r.flags & 16)) dump[i] = dr;
        if (rec) rec[i] = r;
    } else if (consume && rec) {
        gnsship_trk_epoch r = {};
        rec[i] = r;
    }
    c.ran = 0;
    if (emit) {
        const uint64_t vl = k.conf.vector_length;
        const bool runnable = (c.state == 2 || c.state == 3 || c.state == 4) && c.nitems_read >= buf_first &&
                              c.nitems_read + vl <= buf_first + static_cast<uint64_t>(buf_len);
        const int64_t off = static_cast<int64_t>(c.nitems_read - buf_first);
        const float zero[1] = {0.0f};
        for (int q = 0; q < k.jobs_per_channel; q++) {
            const int n_taps = q == 0 ? k.n_taps : 1;
            const float* sh = q == 0 ? (c.narrow ? k.shifts_n : k.shifts) : zero;
            if (hd_jobs) {  // high_dyn: the high-dynamics pair (dll_pll_veml_tracking.cc:530,536)
                HdJob& j = hd_jobs[jb + q];
                if (runnable) {
                    fill_hd_job(j, k, c, off, n_taps, sh);
                } else {
                    j.n_samples = 0;
                }
                for (int m = 0; m < j.n_chunks; m++) {
                    const int rem = static_cast<int>(vl) - m * kCorrChunk;  // HD chunks are kCorrChunk samples too
                    hd_chunks[j.first_chunk + m].len = runnable ? (rem < kCorrChunk ? rem : kCorrChunk) : 0;
                }
                continue;
            }
            DevJob& j = jobs[jb + q];
            if (runnable) {
                fill_job(j, k, c, off, q == 0 ? c.code_id : c.data_code_id, n_taps, sh);
                // the next epoch's rotator anchors, replayed here instead of by a separate anchor
                // launch; the data job shares the pilot job's NCO, hence its anchors
                if (q == 0) {
                    replay_anchors(j, anchors, 0, kAnchorSegments);
                } else {
                    const DevJob& j0 = jobs[jb];
                    const int nblk = (j.n_samples + kRenorm - 1) / kRenorm;
                    for (int b = 0; b < nblk; b++) anchors[j.anchor_offset + b] = anchors[j0.anchor_offset + b];
                }
            } else {
                j.n_samples = 0;
            }
            for (int m = 0; m < k.chunks_per_job; m++) {
                const int start = m * kCorrChunk;
                const int rem = static_cast<int>(vl) - start;
                chunks[j.first_chunk + m].len = runnable ? (rem < kCorrChunk ? rem : kCorrChunk) : 0;
            }
        }
        if (runnable) {
            c.ran = 1;
            c.epoch_start = c.nitems_read;
            atomicAdd(ran_count, 1);
        }
    }
    chans[i] = c;
}

}  // namespace

hipError_t launch_trk_step(const TrkParams* params, TrkChannel* chans, int n_chans, DevJob* jobs, ChunkDesc* chunks, const float* corr_out,
    uint64_t buf_first, int64_t buf_len, int consume, int emit, gnsship_trk_epoch* rec, gnsship_trk_dump_record* dump, int* ran_count,
    TrkHist* hist, HdJob* hd_jobs, HdChunk* hd_chunks, Anchor* anchors, hipStream_t stream)
{
    hipLaunchKernelGGL(trk_step_kernel, dim3((n_chans + 63) / 64), dim3(64), 0, stream, params, chans, n_chans, jobs, chunks, corr_out, buf_first,
        buf_len, consume, emit, rec, dump, ran_count, hist, hd_jobs, hd_chunks, anchors);
    return hipGetLastError();
}

}  // namespace gnsship
