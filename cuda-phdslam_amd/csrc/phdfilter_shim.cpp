/*
 * phdfilter_shim.cpp — the reference's C++ filter API (include/phdfilter.h)
 * on top of the C-ABI.  Part of libphdslam.so.
 *
 * Semantics follow the reference host functions:
 *   setDeviceConfig            phdfilter.cu:3885-3890
 *   initRandomNumberGenerators phdfilter.cu:142-157 (here: reset the RNG contract)
 *   phdPredict                 phdfilter.cu:1080-1257 (incl. n_predict_particles
 *                              duplication and weight down-scaling, :1185-1238)
 *   phdUpdateSynth             phdfilter.cu:3336-3761 (returns the pre-update copy);
 *                              feature_model 2 mirrors maps_dynamic too
 *                              (phdUpdateKernelMixed, predictMapMixed in phdPredict)
 *   recoverSlamState           main.cpp:318-388 (the EAP map, reduceGaussianMixture
 *                              gm_reduce.cpp:59-132, on the device: phd_expected_map)
 *   resampleParticles          main.cpp:453-501 (fixed-point CDF, phd_detmath.h)
 * Like checkCudaErrors in the reference, an unrecoverable error prints and exits.
 * Host-side reads of the configuration use the last setDeviceConfig() value
 * (the reference reads its global `config`, which main.cpp keeps in sync).
 */
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

#include "phd_capi.h"
#include "phd_detmath.h"
#include "phd_rng.h"
#include "phdfilter.h"

namespace {

struct Shim {
    phd_ctx* ctx = nullptr;
    int n = 0;
    phd_capacity cap{};
    SlamConfig cfg{};
    bool cfg_set = false;
    uint64_t seed = 0x5eed5eedULL;
    uint64_t step = 0;
};
Shim g;

[[noreturn]] void die(const char* where) {
    fprintf(stderr, "phdslam: %s failed: %s\n", where, phd_last_error());
    exit(EXIT_FAILURE);
}

void need_config() {
    if (!g.cfg_set) {
        fprintf(stderr, "phdslam: setDeviceConfig() must be called before filtering\n");
        exit(EXIT_FAILURE);
    }
}

/* (Re)create the device context for n particles with room for maps of need_map components. */
void ensure_ctx(int n, int need_map, int grow = 0) {
    if (g.ctx && g.n == n && g.cap.map_capacity >= need_map && !grow) return;
    if (g.ctx) phd_ctx_destroy(g.ctx);
    g.ctx = nullptr;
    int cap = 1024;
    while (cap < need_map) cap *= 2;
    for (int i = 0; i < grow; i++) cap *= 2;
    phd_capacity c{};
    c.map_capacity = cap;
    c.max_measurements = 256;
    c.candidate_capacity = cap + 1024;
    c.survivor_capacity = 1024;
    if (phd_ctx_create(&g.ctx, 0, n, &c) != PHD_OK) die("phd_ctx_create");
    phd_ctx_info(g.ctx, nullptr, &g.cap);
    g.n = n;
    if (phd_set_config(g.ctx, &g.cfg) != PHD_OK) die("phd_set_config");
    phd_set_seed(g.ctx, g.seed);
    // the reference surface adds births explicitly (addBirths, phdfilter.cu.bak:794)
    if (phd_set_step_births(g.ctx, 0) != PHD_OK) die("phd_set_step_births");
}

float safe_log(float x) { return x <= 0 ? -FLT_MAX : std::log(x); }

bool mixed() { return g.cfg.featureModel == MIXED_MODEL; }

/* feature_model 2: the caller's dynamic maps into the context (after
 * phd_load_particles, so particle i owns slab i), room for `extra` more
 * components per particle (the update's births). */
void load_dynamic(const SynthSLAM& particles, int extra) {
    const int n = particles.n_particles;
    vector<int> off(n + 1, 0);
    int need = 0;
    for (int i = 0; i < n; i++) {
        const int sz = (int)particles.maps_dynamic[i].size();
        need = std::max(need, sz);
        off[i + 1] = off[i] + sz;
    }
    int dcap = 256;
    while (dcap < need + extra) dcap *= 2;
    if (phd_enable_dynamic(g.ctx, dcap) != PHD_OK) die("phd_enable_dynamic");
    vector<Gaussian4D> flat((size_t)std::max(off[n], 1));
    for (int i = 0; i < n; i++)
        std::copy(particles.maps_dynamic[i].begin(), particles.maps_dynamic[i].end(), flat.begin() + off[i]);
    if (phd_load_dynamic_maps(g.ctx, n, flat.data(), off.data()) != PHD_OK) die("phd_load_dynamic_maps");
}

void export_dynamic(SynthSLAM& particles) {
    const int n = particles.n_particles;
    vector<int> sizes(n);
    if (phd_dynamic_sizes(g.ctx, sizes.data()) != PHD_OK) die("phd_dynamic_sizes");
    vector<int> off(n + 1, 0);
    for (int i = 0; i < n; i++) off[i + 1] = off[i] + sizes[i];
    vector<Gaussian4D> out((size_t)std::max(off[n], 1));
    if (phd_export_dynamic_maps(g.ctx, n, off.data(), out.data()) != PHD_OK) die("phd_export_dynamic_maps");
    for (int i = 0; i < n; i++) particles.maps_dynamic[i].assign(out.begin() + off[i], out.begin() + off[i + 1]);
}

/* static maps as CSR */
void flatten_static(const SynthSLAM& particles, vector<Gaussian2D>& flat, vector<int>& offsets, int& need) {
    const int n = particles.n_particles;
    offsets.assign(n + 1, 0);
    need = 0;
    for (int i = 0; i < n; i++) {
        const int sz = (int)particles.maps_static[i].size();
        need = std::max(need, sz);
        offsets[i + 1] = offsets[i] + sz;
    }
    flat.resize((size_t)std::max(offsets[n], 1));
    for (int i = 0; i < n; i++)
        std::copy(particles.maps_static[i].begin(), particles.maps_static[i].end(), flat.begin() + offsets[i]);
}

}  // namespace

void setDeviceConfig(const SlamConfig& config) {
    g.cfg = config;
    g.cfg_set = true;
    if (g.ctx && phd_set_config(g.ctx, &g.cfg) != PHD_OK) die("phd_set_config");
}

void initRandomNumberGenerators() {
    const char* s = getenv("PHDSLAM_SEED");
    g.seed = s ? strtoull(s, nullptr, 0) : 0x5eed5eedULL;
    g.step = 0;
    if (g.ctx) phd_set_seed(g.ctx, g.seed);
}

void predictMap(SynthSLAM&) {
    // Declared by the reference but never defined (phdfilter.cu:76); static maps
    // are not predicted and dynamic maps are predicted by phdPredict (feature_model 2).
}

void phdPredict(SynthSLAM& particles, ...) {
    need_config();
    AckermanControl control{0.f, 0.f};
    if (g.cfg.motionType == ACKERMAN_MOTION) {
        va_list ap;
        va_start(ap, particles);
        control = va_arg(ap, AckermanControl);
        va_end(ap);
    }
    const int npp = g.cfg.nPredictParticles > 0 ? g.cfg.nPredictParticles : 1;
    if (npp > 1) {  // duplicate maps, cardinalities, weights (phdfilter.cu:1185-1238)
        SynthSLAM dup(particles.n_particles * npp);
        for (int i = 0; i < particles.n_particles; i++)
            for (int k = 0; k < npp; k++) {
                const int j = i * npp + k;
                dup.states[j] = particles.states[i];
                dup.maps_static[j] = particles.maps_static[i];
                dup.maps_dynamic[j] = particles.maps_dynamic[i];
                dup.cardinalities[j] = particles.cardinalities[i];
                dup.weights[j] = particles.weights[i] - safe_log((float)npp);
                dup.resample_idx[j] = particles.resample_idx[i];
                dup.variances[j] = particles.variances[i];
            }
        particles = dup;
    }
    const int n = particles.n_particles;
    // the device path predicts each (expanded) particle independently
    SlamConfig c1 = g.cfg;
    c1.nPredictParticles = 1;
    if (mixed()) {
        // predictMapMixed runs with the pose predict (phdfilter.cu:1241-1242):
        // both maps into the context, the dynamic ones predicted there
        vector<Gaussian2D> flat;
        vector<int> offsets;
        int need = 0;
        flatten_static(particles, flat, offsets, need);
        ensure_ctx(n, need);
        if (phd_load_particles(g.ctx, n, particles.states.data(), particles.weights.data(), flat.data(),
                               offsets.data()) != PHD_OK)
            die("phd_load_particles");
        load_dynamic(particles, 0);
    } else {
        ensure_ctx(n, 0);
    }
    if (phd_set_config(g.ctx, &c1) != PHD_OK) die("phd_set_config");
    if (phd_set_poses(g.ctx, n, particles.states.data()) != PHD_OK) die("phd_set_poses");
    int rc = (g.cfg.motionType == ACKERMAN_MOTION) ? phd_predict_ackerman(g.ctx, control, nullptr, g.step)
                                                  : phd_predict_cv(g.ctx, nullptr, g.step);
    if (rc != PHD_OK) die("phdPredict");
    g.step++;
    if (phd_export_particles(g.ctx, n, particles.states.data(), nullptr, nullptr) != PHD_OK) die("export");
    if (mixed()) export_dynamic(particles);
    phd_set_config(g.ctx, &g.cfg);
}

SynthSLAM phdUpdateSynth(SynthSLAM& particles, measurementSet measurements) {
    need_config();
    SynthSLAM pre(particles);
    const int n = particles.n_particles;
    int need = 0;
    vector<int> offsets(n + 1, 0);
    for (int i = 0; i < n; i++) {
        const int sz = (int)particles.maps_static[i].size();
        need = std::max(need, sz);
        offsets[i + 1] = offsets[i] + sz;
    }
    vector<Gaussian2D> flat((size_t)std::max(offsets[n], 1));
    for (int i = 0; i < n; i++) std::copy(particles.maps_static[i].begin(), particles.maps_static[i].end(),
                                          flat.begin() + offsets[i]);
    const int M = std::min((int)measurements.size(), 256);
    for (int attempt = 0;; attempt++) {
        ensure_ctx(n, need + 2 * M, attempt);
        if (phd_load_particles(g.ctx, n, particles.states.data(), particles.weights.data(), flat.data(),
                               offsets.data()) != PHD_OK)
            die("phd_load_particles");
        if (mixed()) load_dynamic(particles, 2 * M);
        if (phd_set_measurements(g.ctx, measurements.data(), M) != PHD_OK) die("phd_set_measurements");
        const int rc = phd_update(g.ctx);
        if (rc == PHD_E_CAPACITY && attempt < 3) continue;
        if (rc != PHD_OK) die("phdUpdateSynth");
        break;
    }
    if (phd_normalize(g.ctx, nullptr) != PHD_OK) die("phd_normalize");
    vector<int> sizes(n);
    if (phd_export_particles(g.ctx, n, nullptr, particles.weights.data(), sizes.data()) != PHD_OK) die("export");
    vector<int> oo(n + 1, 0);
    for (int i = 0; i < n; i++) oo[i + 1] = oo[i] + sizes[i];
    vector<Gaussian2D> out((size_t)std::max(oo[n], 1));  // (an empty store still needs a buffer)
    if (phd_export_maps(g.ctx, n, oo.data(), out.data()) != PHD_OK) die("export maps");
    for (int i = 0; i < n; i++) particles.maps_static[i].assign(out.begin() + oo[i], out.begin() + oo[i + 1]);
    if (mixed()) export_dynamic(particles);
    if (g.cfg.filterType == CPHD_TYPE) {
        // the posterior log cardinality distribution of every particle
        // (phdfilter.cu.bak:2700-2706: particles.cardinalities[i] = cn_update row i)
        const int K = g.cfg.maxCardinality + 1;
        vector<float> cn((size_t)n * K);
        if (phd_cardinality_distribution(g.ctx, cn.data()) != PHD_OK) die("phd_cardinality_distribution");
        for (int i = 0; i < n; i++) particles.cardinalities[i].assign(cn.begin() + (size_t)i * K, cn.begin() + (size_t)(i + 1) * K);
    }
    return pre;
}

void addBirths(SynthSLAM& particles, measurementSet measurements) {
    need_config();
    const int n = particles.n_particles;
    const int M = std::min((int)measurements.size(), 256);
    if (M == 0) return;
    int need = 0;
    vector<int> offsets(n + 1, 0);
    for (int i = 0; i < n; i++) {
        const int sz = (int)particles.maps_static[i].size();
        need = std::max(need, sz);
        offsets[i + 1] = offsets[i] + sz;
    }
    vector<Gaussian2D> flat((size_t)std::max(offsets[n], 1));
    for (int i = 0; i < n; i++)
        std::copy(particles.maps_static[i].begin(), particles.maps_static[i].end(), flat.begin() + offsets[i]);
    ensure_ctx(n, need + M + 2 * M);
    if (phd_load_particles(g.ctx, n, particles.states.data(), particles.weights.data(), flat.data(),
                           offsets.data()) != PHD_OK)
        die("phd_load_particles");
    if (phd_add_births(g.ctx, measurements.data(), M) != PHD_OK) die("phd_add_births");
    vector<int> sizes(n);
    if (phd_export_particles(g.ctx, n, nullptr, nullptr, sizes.data()) != PHD_OK) die("export");
    vector<int> oo(n + 1, 0);
    for (int i = 0; i < n; i++) oo[i + 1] = oo[i] + sizes[i];
    vector<Gaussian2D> out((size_t)std::max(oo[n], 1));
    if (phd_export_maps(g.ctx, n, oo.data(), out.data()) != PHD_OK) die("export maps");
    for (int i = 0; i < n; i++) particles.maps_static[i].assign(out.begin() + oo[i], out.begin() + oo[i + 1]);
}

void recoverSlamState(SynthSLAM& particles, ConstantVelocityState& expectedPose, vector<REAL>& cn_estimate) {
    if (particles.n_particles > 1) {
        double e[6] = {0, 0, 0, 0, 0, 0};
        for (int i = 0; i < particles.n_particles; i++) {
            const float ew = std::exp(particles.weights[i]);
            const float* s = &particles.states[i].px;
            for (int k = 0; k < 6; k++) e[k] += (double)(ew * s[k]);
        }
        float* ep = &expectedPose.px;
        for (int k = 0; k < 6; k++) ep[k] = (float)e[k];
        if (g.cfg.mapEstimate & 1) {
            float mw = -FLT_MAX;
            int mi = 0;
            for (int i = 0; i < particles.n_particles; i++)
                if (particles.weights[i] > mw) {
                    mw = particles.weights[i];
                    mi = i;
                }
            particles.max_map_static = particles.maps_static[mi];
            particles.max_map_dynamic = particles.maps_dynamic[mi];
            cn_estimate = particles.cardinalities[mi];
        }
        if (g.cfg.mapEstimate & 2) {
            // EAP map on the device (phd_expected_map, phd_eap.hip): the caller's
            // particles are loaded into the shim's context, reduced there, read back
            const int n = particles.n_particles;
            vector<int> offsets(n + 1, 0);
            int need = 0;
            for (int i = 0; i < n; i++) {
                const int sz = (int)particles.maps_static[i].size();
                need = std::max(need, sz);
                offsets[i + 1] = offsets[i] + sz;
            }
            vector<Gaussian2D> flat((size_t)std::max(offsets[n], 1));
            for (int i = 0; i < n; i++)
                std::copy(particles.maps_static[i].begin(), particles.maps_static[i].end(), flat.begin() + offsets[i]);
            ensure_ctx(n, need);
            if (phd_load_particles(g.ctx, n, particles.states.data(), particles.weights.data(), flat.data(),
                                   offsets.data()) != PHD_OK)
                die("phd_load_particles");
            long nout = 0;
            vector<Gaussian2D> out((size_t)std::max(offsets[n], 1));
            if (phd_expected_map(g.ctx, out.data(), (long)offsets[n], &nout) != PHD_OK) die("phd_expected_map");
            out.resize((size_t)nout);
            particles.exp_map_static = out;
            // exp_map_dynamic (main.cpp:369-371): the dynamic maps, reduced the same way
            particles.exp_map_dynamic.clear();
            if (mixed()) {
                load_dynamic(particles, 0);
                long ndyn = 0;
                size_t tot = 0;
                for (int i = 0; i < n; i++) tot += particles.maps_dynamic[i].size();
                vector<Gaussian4D> dout(std::max<size_t>(tot, 1));
                if (phd_expected_map_dynamic(g.ctx, dout.data(), (long)tot, &ndyn) != PHD_OK)
                    die("phd_expected_map_dynamic");
                dout.resize((size_t)ndyn);
                particles.exp_map_dynamic = dout;
            }
            // main.cpp:372-378 clears cn_estimate and then loops over its (zero)
            // entries, so writeLog reads past the end of an empty vector.  Here:
            // the intended expression, Σ_i exp(w_i) cardinalities[i][j].
            cn_estimate.clear();
            if (!particles.cardinalities.empty() && !particles.cardinalities[0].empty()) {
                cn_estimate.assign(particles.cardinalities[0].size(), 0.f);
                for (int i = 0; i < n; i++) {
                    const float ew = std::exp(particles.weights[i]);
                    const vector<REAL>& ci = particles.cardinalities[i];
                    for (size_t j = 0; j < cn_estimate.size() && j < ci.size(); j++) cn_estimate[j] += ew * ci[j];
                }
            }
        }
    } else {
        expectedPose = particles.states[0];
        particles.max_map_static = particles.maps_static[0];
        particles.max_map_dynamic = particles.maps_dynamic[0];
        cn_estimate = particles.cardinalities[0];
    }
}

SynthSLAM resampleParticles(const SynthSLAM& particles, int n_new, uint64_t step) {
    const int n = particles.n_particles;
    if (n_new < 0) n_new = n;
    vector<uint64_t> cdf(n);
    uint64_t acc = 0;
    float tmax = -1.f;
    int amax = 0;
    for (int i = 0; i < n; i++) {
        const float t = phd_det_expf(particles.weights[i]);
        acc += phd_fix_term(t);
        cdf[i] = acc;
        if (t > tmax) {
            tmax = t;
            amax = i;
        }
    }
    vector<int> idx(n_new);
    for (int j = 0; j < n_new; j++) {
        const phd_u32x4 x = phd_rng_draw(g.seed, (uint32_t)j, step, PHD_STREAM_RESAMPLE);
        const uint64_t r = phd_fix_stratum(j, phd_u01(x.v[0]), n_new);
        const int k = (int)(std::lower_bound(cdf.begin(), cdf.end(), r) - cdf.begin());
        idx[j] = k < n ? k : amax;
    }
    return particles.copy_particles(idx);
}
