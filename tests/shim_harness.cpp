/*
 * shim_harness.cpp — test driver for the C++ drop-in surface (include/phdfilter.h).
 * Built by cuda-phdslam_amd/build.py into tests/shim_harness; used only by
 * tests/test_gpu_parity.py to hold phdPredict / addBirths / phdUpdateSynth, as a
 * reference-style caller uses them (main.cpp:1178-1312), against the oracle.
 *
 *   shim_harness <in.bin> <out.bin>
 *
 * in.bin (little endian): int32 ops (1 predict, 2 addBirths(Zb), 4 phdUpdateSynth(Z)),
 *   int32 n, int32 M, int32 Mb, uint64 seed, SlamConfig (324 B), AckermanControl (8 B),
 *   ConstantVelocityState[n], float logw[n], int32 sizes[n], Gaussian2D[sum sizes],
 *   RangeBearingMeasurement[M], RangeBearingMeasurement[Mb]
 * out.bin: int32 n, int32 K, ConstantVelocityState[n], float logw[n],
 *   int32 sizes[n], Gaussian2D[sum sizes], float cardinalities[n*K]
 * feature_model 2 (mixed): in.bin continues with int32 dsizes[n],
 *   Gaussian4D[sum dsizes]; out.bin ends with int32 dsizes[n], Gaussian4D[...].
 */
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "phdfilter.h"

template <class T>
static void rd(FILE* f, T* p, size_t n) {
    if (n && fread(p, sizeof(T), n, f) != n) {
        fprintf(stderr, "shim_harness: short input\n");
        exit(2);
    }
}

template <class T>
static void wr(FILE* f, const T* p, size_t n) {
    if (n) fwrite(p, sizeof(T), n, f);
}

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s <in.bin> <out.bin>\n", argv[0]);
        return 1;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    int32_t hdr[4];
    uint64_t seed;
    SlamConfig cfg;
    AckermanControl u;
    rd(f, hdr, 4);
    rd(f, &seed, 1);
    rd(f, &cfg, 1);
    rd(f, &u, 1);
    const int ops = hdr[0], n = hdr[1], M = hdr[2], Mb = hdr[3];
    SynthSLAM particles((unsigned)n);
    rd(f, particles.states.data(), n);
    rd(f, particles.weights.data(), n);
    std::vector<int32_t> sizes(n);
    rd(f, sizes.data(), n);
    for (int i = 0; i < n; i++) {
        particles.maps_static[i].resize(sizes[i]);
        rd(f, particles.maps_static[i].data(), sizes[i]);
    }
    measurementSet Z(M), Zb(Mb);
    rd(f, Z.data(), M);
    rd(f, Zb.data(), Mb);
    const bool mixed = cfg.featureModel == MIXED_MODEL;
    if (mixed) {
        std::vector<int32_t> dsz(n);
        rd(f, dsz.data(), n);
        for (int i = 0; i < n; i++) {
            particles.maps_dynamic[i].resize(dsz[i]);
            rd(f, particles.maps_dynamic[i].data(), dsz[i]);
        }
    }
    fclose(f);

    setenv("PHDSLAM_SEED", std::to_string(seed).c_str(), 1);
    setDeviceConfig(cfg);
    initRandomNumberGenerators();
    if (ops & 1) phdPredict(particles, u);
    if (ops & 2) addBirths(particles, Zb);
    if (ops & 4) phdUpdateSynth(particles, Z);

    FILE* o = fopen(argv[2], "wb");
    if (!o) return 1;
    const int32_t nn = particles.n_particles;
    const int32_t K = (nn > 0 && !particles.cardinalities[0].empty()) ? (int32_t)particles.cardinalities[0].size() : 0;
    wr(o, &nn, 1);
    wr(o, &K, 1);
    wr(o, particles.states.data(), nn);
    wr(o, particles.weights.data(), nn);
    for (int i = 0; i < nn; i++) {
        const int32_t s = (int32_t)particles.maps_static[i].size();
        wr(o, &s, 1);
    }
    for (int i = 0; i < nn; i++) wr(o, particles.maps_static[i].data(), particles.maps_static[i].size());
    for (int i = 0; i < nn; i++) wr(o, particles.cardinalities[i].data(), (size_t)K);
    if (mixed) {
        for (int i = 0; i < nn; i++) {
            const int32_t s = (int32_t)particles.maps_dynamic[i].size();
            wr(o, &s, 1);
        }
        for (int i = 0; i < nn; i++) wr(o, particles.maps_dynamic[i].data(), particles.maps_dynamic[i].size());
    }
    fclose(o);
    return 0;
}
