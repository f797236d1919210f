/*
 * phdslam_run.cpp — the run_synth driver (main.cpp:1075-1322) rebuilt on the
 * drop-in API (include/phdfilter.h) or, with --device-loop, on the
 * device-resident C-ABI loop (phd_step).
 *
 *   phdslam_run <config.cfg> [--data DIR] [--steps N] [--triples] [--header]
 *               [--log DIR] [--device-loop]
 *
 * Inputs (DATA = data_directory of the cfg, or --data), read by the
 * reference-format loaders of include/phd_io.h (main.cpp:147-245):
 *   DATA/measurements.txt  one time step per line, range/bearing pairs
 *                          (--triples: range bearing label, the format
 *                          parseMeasurements reads, main.cpp:190-205)
 *   DATA/controls.txt      one "v_encoder alpha" per line (',' separators accepted)
 * Lines starting with '%' or '#' are comments; --header skips the first line of
 * each file as the reference's loaders do.  Step n uses measurements[n] and,
 * for n > 0, controls[n-1] (main.cpp:1233-1234).
 * --log DIR writes DIR/state_estimateNNNNN.log every step (writeLog,
 * main.cpp:848-954): expected pose, the EAP (mapEstimate & 2) or MAP map,
 * log-weights, poses, resample indices, cardinality.
 *
 *   phdslam_run --synth C [--gpus N] [--particles P] [--steps K] [--replay]
 *               [--block-records R] [--resample-every] [--dump FILE]
 *
 * Multi-GPU without PyTorch (include/phd_group.h): one
 * process drives N GPUs, each holding a P-particle shard of ONE filter on the
 * synthetic scenario of BASELINE config C (phd_synth_*, every shard the same
 * prior as bench.py's ranks), through RCCL (ncclCommInitAll, grouped calls):
 * the sharded step of phdslam/dist.py.  --replay times K steps of the bench's
 * replay workload and prints steps/s; --dump writes every shard's final state
 * (poses, log-weights, map sizes, maps; rank order) for the parity test.
 */
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "phd_capi.h"
#include "phd_group.h"
#include "phd_io.h"
#include "phdfilter.h"

static std::vector<AckermanControl> load_controls(const std::string& path, int flags) {
    int n = 0;
    phd_load_controls(path.c_str(), flags, nullptr, 0, &n);
    std::vector<AckermanControl> u((size_t)n);
    if (n > 0 && phd_load_controls(path.c_str(), flags, u.data(), n, &n) != PHD_OK) u.clear();
    return u;
}

static std::vector<measurementSet> load_measurements(const std::string& path, int flags) {
    int steps = 0, off0 = 0;
    phd_load_measurements(path.c_str(), flags, nullptr, 0, &off0, 0, &steps);
    std::vector<int> offs((size_t)steps + 1, 0);
    phd_load_measurements(path.c_str(), flags, nullptr, 0, offs.data(), steps, &steps);
    std::vector<RangeBearingMeasurement> z((size_t)offs[steps]);
    std::vector<measurementSet> all;
    if (phd_load_measurements(path.c_str(), flags, z.data(), (long)z.size(), offs.data(), steps, &steps) != PHD_OK)
        return all;
    for (int s = 0; s < steps; s++) all.emplace_back(z.begin() + offs[s], z.begin() + offs[s + 1]);
    return all;
}

/* bench.py's capacities (phdslam.scenario.bench_capacities, the tight set) */
static phd_capacity synth_capacities(int cid, int G, int M) {
    phd_capacity cap{};
    cap.map_capacity = (G + 2 * M + 64 + 63) / 64 * 64;
    cap.max_measurements = M;
    cap.candidate_capacity = cid == 5 ? 1800 : cid == 4 ? G + 4 * M + 16 : G + 3 * M + (cid == 3 ? 0 : 16);
    cap.survivor_capacity = cid == 5 ? 640 : 3 * M + 32;
    return cap;
}

static int run_synth_sharded(int argc, char** argv) {
    int cid = 3, world = 1, P = 0, steps = 10, K = 4;
    bool replay = false, every = false;
    std::string dump;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--synth") && i + 1 < argc) cid = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) world = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--particles") && i + 1 < argc) P = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--steps") && i + 1 < argc) steps = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--block-records") && i + 1 < argc) K = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--dump") && i + 1 < argc) dump = argv[++i];
        else if (!strcmp(argv[i], "--replay")) replay = true;
        else if (!strcmp(argv[i], "--resample-every")) every = true;
    }
    SlamConfig cfg;
    int n0 = 0, G = 0, M = 0;
    float df = 0.f;
    if (phd_synth_preset(cid, &cfg, &n0, &G, &M, &df) != PHD_OK) {
        fprintf(stderr, "phd_synth_preset(%d): %s\n", cid, phd_last_error());
        return 1;
    }
    if (cid == 4 && !P) n0 /= world > 0 ? world : 1;  // config 4: the 32768-particle job split over the GPUs
    const int n = P ? P : n0;
    if (every) cfg.resampleThresh = 1.0f;
    int ndev = 0;
    phd_device_count(&ndev);
    if (world < 1 || world > ndev) {
        fprintf(stderr, "--gpus %d: %d HIP devices visible\n", world, ndev);
        return 1;
    }
    const uint64_t seed = 20261015ULL + (uint64_t)cid;  // phdslam.scenario.SEED_BASE + config (bench.py)
    std::vector<ConstantVelocityState> poses((size_t)n);
    std::vector<float> lw((size_t)n);
    std::vector<Gaussian2D> maps((size_t)n * G);
    std::vector<int> offs((size_t)n + 1);
    std::vector<RangeBearingMeasurement> z((size_t)M);
    if (phd_synth_scenario(&cfg, n, G, M, df, seed, poses.data(), lw.data(), maps.data(), offs.data(), z.data()) !=
        PHD_OK) {
        fprintf(stderr, "phd_synth_scenario: %s\n", phd_last_error());
        return 1;
    }
    const phd_capacity cap = synth_capacities(cid, G, M);
    std::vector<phd_ctx*> ctx((size_t)world, nullptr);
    std::vector<int> devs((size_t)world);
    for (int r = 0; r < world; r++) {
        devs[r] = r;
        if (phd_ctx_create(&ctx[r], r, n, &cap) != PHD_OK || phd_set_config(ctx[r], &cfg) != PHD_OK ||
            phd_set_seed(ctx[r], seed) != PHD_OK ||
            phd_load_particles(ctx[r], n, poses.data(), lw.data(), maps.data(), offs.data()) != PHD_OK ||
            phd_set_measurements(ctx[r], z.data(), M) != PHD_OK || (replay && phd_set_replay(ctx[r], 1) != PHD_OK) ||
            phd_set_check_each_update(ctx[r], 0) != PHD_OK) {
            fprintf(stderr, "rank %d: %s\n", r, phd_last_error());
            return 1;
        }
    }
    phd_group* g = nullptr;
    if (phd_group_create(&g, world, ctx.data(), devs.data(), K, 0x9e3779b97f4a7c15ULL) != PHD_OK) {
        fprintf(stderr, "phd_group_create: %s\n", phd_group_last_error());
        return 1;
    }
    const phd_ackerman_control u{0.05f, 2.0f};  // (alpha, v_encoder): bench.py's control (2.0, 0.05)
    const phd_ackerman_control* up = cfg.motionType == CV_MOTION ? nullptr : &u;
    const int warm = replay ? 10 : 0;
    for (int k = 0; k < warm; k++)
        if (phd_group_step(g, up, (uint64_t)k, nullptr, nullptr) != PHD_OK) {
            fprintf(stderr, "step %d: %s\n", k, phd_group_last_error());
            return 1;
        }
    if (phd_group_flush(g) != PHD_OK) {
        fprintf(stderr, "flush: %s\n", phd_group_last_error());
        return 1;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < steps; k++) {
        const uint64_t sk = replay ? (uint64_t)(warm + k) : (uint64_t)(k + 1);
        if (phd_group_step(g, up, sk, nullptr, nullptr) != PHD_OK) {
            fprintf(stderr, "step %d: %s\n", k, phd_group_last_error());
            return 1;
        }
    }
    if (phd_group_flush(g) != PHD_OK) {
        fprintf(stderr, "flush: %s\n", phd_group_last_error());
        return 1;
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    long long st[5];
    phd_group_stats(g, st);
    for (int r = 0; r < world; r++)
        if (phd_check_errors(ctx[r]) != PHD_OK) {
            fprintf(stderr, "rank %d: %s\n", r, phd_last_error());
            return 1;
        }
    printf("{\"config\": %d, \"gpus\": %d, \"particles_per_gpu\": %d, \"steps\": %d, \"mode\": \"%s\", "
           "\"steps_per_s\": %.2f, \"ms_per_step\": %.4f, \"resamples\": %lld, \"migrated\": %lld, "
           "\"records\": %lld, \"overflow_records\": %lld, \"pending_slots\": %lld}\n",
           cid, world, n, steps, replay ? "replay" : "sequence", steps / secs, 1e3 * secs / steps, st[0], st[1], st[2],
           st[3], st[4]);
    if (!dump.empty()) {
        FILE* fp = fopen(dump.c_str(), "wb");
        if (!fp) {
            fprintf(stderr, "cannot write %s\n", dump.c_str());
            return 1;
        }
        for (int r = 0; r < world; r++) {
            std::vector<ConstantVelocityState> ps((size_t)n);
            std::vector<float> w((size_t)n);
            std::vector<int> sz((size_t)n), oo((size_t)n + 1, 0);
            if (phd_export_particles(ctx[r], n, ps.data(), w.data(), sz.data()) != PHD_OK) {
                fprintf(stderr, "export: %s\n", phd_last_error());
                return 1;
            }
            for (int i = 0; i < n; i++) oo[i + 1] = oo[i] + sz[i];
            std::vector<Gaussian2D> mm((size_t)std::max(oo[n], 1));
            if (phd_export_maps(ctx[r], n, oo.data(), mm.data()) != PHD_OK) {
                fprintf(stderr, "export: %s\n", phd_last_error());
                return 1;
            }
            fwrite(&n, sizeof(int), 1, fp);
            fwrite(ps.data(), sizeof(ConstantVelocityState), (size_t)n, fp);
            fwrite(w.data(), sizeof(float), (size_t)n, fp);
            fwrite(sz.data(), sizeof(int), (size_t)n, fp);
            fwrite(mm.data(), sizeof(Gaussian2D), (size_t)oo[n], fp);
        }
        fclose(fp);
    }
    phd_group_destroy(g);
    for (phd_ctx* c : ctx) phd_ctx_destroy(c);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && !strcmp(argv[1], "--synth")) return run_synth_sharded(argc, argv);
    if (argc < 2) {
        fprintf(stderr, "usage: %s <config.cfg> [--data DIR] [--steps N] [--triples] [--device-loop]\n", argv[0]);
        return 1;
    }
    SlamConfig config;
    char data_dir[4096] = "";
    if (phd_config_load(argv[1], &config, data_dir, sizeof(data_dir)) != PHD_OK) {
        fprintf(stderr, "Unable to load config file: %s\n", argv[1]);
        return 1;
    }
    std::string data = data_dir;
    int n_steps = -1;
    bool triples = false, device_loop = false, header = false;
    std::string log_dir;
    for (int i = 2; i < argc; i++) {
        if (!strcmp(argv[i], "--data") && i + 1 < argc) data = argv[++i];
        else if (!strcmp(argv[i], "--steps") && i + 1 < argc) n_steps = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--log") && i + 1 < argc) log_dir = argv[++i];
        else if (!strcmp(argv[i], "--triples")) triples = true;
        else if (!strcmp(argv[i], "--header")) header = true;
        else if (!strcmp(argv[i], "--device-loop")) device_loop = true;
    }
    if (!data.empty() && data.back() != '/') data += '/';
    const int base_flags = PHD_IO_COMMAS | PHD_IO_COMMENTS | (header ? PHD_IO_HEADER : 0);
    const auto allZ = load_measurements(data + "measurements.txt", base_flags | (triples ? 0 : PHD_IO_PAIRS));
    const auto allU = load_controls(data + "controls.txt", base_flags);
    int nSteps = (int)allZ.size();
    if (n_steps > 0 && n_steps < nSteps) nSteps = n_steps;
    printf("loaded %zu measurement steps, %zu controls; running %d steps with %d particles\n", allZ.size(),
           allU.size(), nSteps, config.n_particles);

    setDeviceConfig(config);
    initRandomNumberGenerators();
    const int N = config.n_particles;
    SynthSLAM particles(N);
    for (int n = 0; n < N; n++) {
        ConstantVelocityState& s = particles.states[n];
        s.px = config.x0;
        s.py = config.y0;
        s.ptheta = config.yaw0;
        s.vx = config.vx0;
        s.vy = config.vy0;
        s.vtheta = config.vyaw0;
    }
    particles.weights.assign(N, -log((float)N));

    auto t0 = std::chrono::steady_clock::now();
    if (!device_loop) {
        ConstantVelocityState expectedPose;
        vector<REAL> cn;
        for (int n = 0; n < nSteps; n++) {
            const measurementSet& ZZ = allZ[n];
            AckermanControl u{0.f, 0.f};
            if (n > 0 && n - 1 < (int)allU.size()) u = allU[n - 1];
            if (n > 0)
                for (int i = 0; i < config.subdividePredict; i++) {
                    if (config.motionType == CV_MOTION)
                        phdPredict(particles);
                    else
                        phdPredict(particles, u);
                }
            // CPHD: births through the prediction from the previous scan
            if (config.filterType == CPHD_TYPE && n > 0 && !allZ[n - 1].empty()) addBirths(particles, allZ[n - 1]);
            if (!ZZ.empty()) phdUpdateSynth(particles, ZZ);
            recoverSlamState(particles, expectedPose, cn);
            float nEff = 0;
            for (int i = 0; i < particles.n_particles; i++) nEff += exp(2 * particles.weights[i]);
            nEff = 1.0 / nEff / particles.n_particles;
            size_t ncomp = 0;
            for (const auto& m : particles.maps_static) ncomp += m.size();
            printf("step %5d |Z|=%3zu nEff=%.4f pose=(%.3f, %.3f, %.4f) mean map size %.1f\n", n, ZZ.size(), nEff,
                   expectedPose.px, expectedPose.py, expectedPose.ptheta, (double)ncomp / particles.n_particles);
            // (main.cpp:1286: also when n_predict_particles > 1 grew the set beyond 5 x n_particles)
            const bool resample = (nEff <= config.resampleThresh && !ZZ.empty()) || particles.n_particles > 5 * N;
            SynthSLAM resampled = resample ? resampleParticles(particles, N, (uint64_t)n) : SynthSLAM(0);
            if (!resample)
                for (int i = 0; i < particles.n_particles; i++) particles.resample_idx[i] = i;  // main.cpp:1291-1296
            if (!log_dir.empty()) {  // writeLog (main.cpp:848-954): this step's estimate, weights and poses
                                     // before the resample, and the resample's parent indices
                const vector<Gaussian2D>& map =
                    (config.mapEstimate & 2) ? particles.exp_map_static : particles.max_map_static;
                const bool has_cn = config.filterType == CPHD_TYPE && (int)cn.size() >= config.maxCardinality + 1;
                // parents of the n_particles children; -1 past them when the live set was larger
                vector<int> idx = resample ? resampled.resample_idx : particles.resample_idx;
                idx.resize((size_t)particles.n_particles, -1);
                if (phd_write_state_log(log_dir.c_str(), n, &expectedPose, map.data(), (long)map.size(),
                                        particles.weights.data(), particles.states.data(), particles.n_particles,
                                        idx.data(), has_cn ? cn.data() : nullptr, config.maxCardinality,
                                        has_cn ? 1 : 0, 1) != PHD_OK) {
                    fprintf(stderr, "cannot write the state log in %s\n", log_dir.c_str());
                    return 1;
                }
            }
            if (resample) particles = resampled;
            if (std::isnan(nEff)) {
                printf("nan weights detected! exiting...\n");
                break;
            }
        }
    } else {
        phd_ctx* ctx = nullptr;
        phd_capacity cap{};
        cap.map_capacity = 1024;
        cap.candidate_capacity = 2048;
        if (config.nPredictParticles > 1) {  // live set: up to npp^subdivide x (5 x n_particles)
            long m = 5L * N;
            for (int k = 0; k < std::max(config.subdividePredict, 1); k++) m *= config.nPredictParticles;
            cap.max_particles = (int)std::min(m, 1L << 24);
        }
        if (phd_ctx_create(&ctx, 0, N, &cap) != PHD_OK || phd_set_config(ctx, &config) != PHD_OK) {
            fprintf(stderr, "phd_ctx_create: %s\n", phd_last_error());
            return 1;
        }
        std::vector<int> offs(N + 1, 0);
        if (phd_load_particles(ctx, N, particles.states.data(), particles.weights.data(), nullptr, offs.data()) !=
            PHD_OK) {
            fprintf(stderr, "phd_load_particles: %s\n", phd_last_error());
            return 1;
        }
        const char* seed_env = getenv("PHDSLAM_SEED");  // the shim's seed (initRandomNumberGenerators)
        phd_set_seed(ctx, seed_env ? strtoull(seed_env, nullptr, 0) : 0x5eed5eedULL);
        const bool cphd = config.filterType == CPHD_TYPE;
        const int K = config.maxCardinality + 1;
        std::vector<ConstantVelocityState> st((size_t)N);
        std::vector<float> w((size_t)N), cn_all, cn;
        std::vector<int> sz((size_t)N), idx((size_t)N);
        for (int n = 0; n < nSteps; n++) {
            AckermanControl u{0.f, 0.f};
            if (n > 0 && n - 1 < (int)allU.size()) u = allU[n - 1];
            const int M = (int)allZ[n].size();
            // the shim's order (main.cpp:1240-1297): predict (sub-steps numbered
            // (n-1)*subdivide + k, as the shim counts its phdPredict calls), update,
            // normalise; then the estimates and the log of the pre-resample state,
            // then the resample with the parents logged
            // (CPHD: the step places the births of the previous scan itself, after
            // the predict and before the update: phd_set_step_births, on by default)
            bool ok = phd_set_measurements(ctx, allZ[n].data(), M) == PHD_OK &&
                      phd_predict_update(ctx, &u, n > 0, n > 0 ? (uint64_t)(n - 1) : 0, nullptr) == PHD_OK;
            int nl = N;  // live particles (n_predict_particles > 1 multiplies them per predict)
            ok = ok && phd_ctx_info(ctx, &nl, nullptr) == PHD_OK;
            st.resize((size_t)nl);
            w.resize((size_t)nl);
            sz.resize((size_t)nl);
            idx.resize((size_t)std::max(nl, N));
            if (!ok ||
                (M > 0 && phd_normalize(ctx, nullptr) != PHD_OK) ||
                phd_export_particles(ctx, nl, st.data(), w.data(), sz.data()) != PHD_OK) {
                fprintf(stderr, "step %d: %s\n", n, phd_last_error());
                return 1;
            }
            float nEff = 0;
            for (int i = 0; i < nl; i++) nEff += exp(2 * w[i]);
            nEff = 1.0 / nEff / nl;
            const bool resample = (nEff <= config.resampleThresh && M > 0) || nl > 5 * N;  // main.cpp:1286
            if (!log_dir.empty()) {  // writeLog from the device store
                ConstantVelocityState ep;
                int mi = 0;
                if (phd_expected_pose(ctx, &ep, &mi) != PHD_OK) {
                    fprintf(stderr, "step %d: %s\n", n, phd_last_error());
                    return 1;
                }
                if (nl == 1) ep = st[0];
                std::vector<Gaussian2D> map;
                long nout = 0;
                if (config.mapEstimate & 2) {  // EAP map on the device
                    long total = 0;
                    for (int i = 0; i < nl; i++) total += sz[i];
                    map.resize((size_t)std::max(total, 1L));
                    if (phd_expected_map(ctx, map.data(), total, &nout) != PHD_OK) {
                        fprintf(stderr, "step %d: %s\n", n, phd_last_error());
                        return 1;
                    }
                } else {  // MAP: the first highest-weight particle's map
                    std::vector<int> oo(nl + 1, 0);
                    for (int i = 0; i < nl; i++) oo[i + 1] = oo[i] + sz[i];
                    std::vector<Gaussian2D> all((size_t)std::max(oo[nl], 1));
                    if (phd_export_maps(ctx, nl, oo.data(), all.data()) != PHD_OK) {
                        fprintf(stderr, "step %d: %s\n", n, phd_last_error());
                        return 1;
                    }
                    map.assign(all.begin() + oo[mi], all.begin() + oo[mi + 1]);
                    nout = (long)map.size();
                }
                bool has_cn = false;
                if (cphd) {
                    cn_all.resize((size_t)nl * K);
                    if (phd_cardinality_distribution(ctx, cn_all.data()) == PHD_OK) {  // fails before any CPHD update
                        // recoverSlamState's rule (as the shim): EAP -> Σ exp(w_i) cn_i, else the MAP particle's
                        cn.assign((size_t)K, 0.f);
                        for (int i = 0; i < nl; i++) {
                            if ((config.mapEstimate & 2) && nl > 1) {
                                const float ew = exp(w[i]);
                                for (int j = 0; j < K; j++) cn[j] += ew * cn_all[(size_t)i * K + j];
                            } else if (i == mi) {
                                for (int j = 0; j < K; j++) cn[j] = cn_all[(size_t)i * K + j];
                            }
                        }
                        has_cn = true;
                    }
                }
                if (resample) {
                    if (phd_resample(ctx, nullptr, (uint64_t)n, idx.data()) != PHD_OK) {
                        fprintf(stderr, "step %d: %s\n", n, phd_last_error());
                        return 1;
                    }
                    for (int i = N; i < nl; i++) idx[i] = -1;  // parents of the n_particles children
                } else {
                    for (int i = 0; i < nl; i++) idx[i] = i;
                }
                if (phd_write_state_log(log_dir.c_str(), n, &ep, map.data(), nout, w.data(), st.data(), nl, idx.data(),
                                        has_cn ? cn.data() : nullptr, config.maxCardinality, has_cn ? 1 : 0,
                                        1) != PHD_OK) {
                    fprintf(stderr, "step %d: %s\n", n, phd_last_error());
                    return 1;
                }
            } else if (resample && phd_resample(ctx, nullptr, (uint64_t)n, nullptr) != PHD_OK) {
                fprintf(stderr, "step %d: %s\n", n, phd_last_error());
                return 1;
            }
        }
        ConstantVelocityState ep;
        int mi;
        phd_expected_pose(ctx, &ep, &mi);
        printf("final expected pose (%.3f, %.3f, %.4f), MAP particle %d\n", ep.px, ep.py, ep.ptheta, mi);
        phd_ctx_destroy(ctx);
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("%d steps in %.3f s (%.1f steps/s)\n", nSteps, secs, nSteps / secs);
    return 0;
}
