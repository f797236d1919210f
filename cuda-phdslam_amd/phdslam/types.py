"""Host-side mirrors of the reference's POD types (include/phd_types.h).

numpy structured dtypes for array data (Gaussian2D, ConstantVelocityState,
RangeBearingMeasurement, ...) and a ctypes Structure for SlamConfig, all
byte-identical to the reference layouts (src/slamtypes.h:44-250).
"""
import ctypes

import numpy as np

GAUSSIAN2D = np.dtype([("cov", np.float32, (4,)), ("mean", np.float32, (2,)), ("weight", np.float32)])
GAUSSIAN4D = np.dtype([("cov", np.float32, (16,)), ("mean", np.float32, (4,)), ("weight", np.float32)])
POSE = np.dtype([("px", np.float32), ("py", np.float32), ("ptheta", np.float32),
                 ("vx", np.float32), ("vy", np.float32), ("vtheta", np.float32)])
ACKERMAN_CONTROL = np.dtype([("alpha", np.float32), ("v_encoder", np.float32)])
ACKERMAN_NOISE = np.dtype([("n_alpha", np.float32), ("n_encoder", np.float32)])
CV_NOISE = np.dtype([("ax", np.float32), ("ay", np.float32), ("atheta", np.float32)])
MEASUREMENT = np.dtype([("range", np.float32), ("bearing", np.float32), ("label", np.int32)])

assert GAUSSIAN2D.itemsize == 28 and POSE.itemsize == 24 and MEASUREMENT.itemsize == 12

MOTION_CV = 0
MOTION_ACKERMAN = 1


class AckermanControl(ctypes.Structure):
    _fields_ = [("alpha", ctypes.c_float), ("v_encoder", ctypes.c_float)]


class Capacity(ctypes.Structure):
    _fields_ = [("map_capacity", ctypes.c_int), ("max_measurements", ctypes.c_int),
                ("candidate_capacity", ctypes.c_int), ("survivor_capacity", ctypes.c_int),
                ("max_particles", ctypes.c_int)]


_f = ctypes.c_float
_i = ctypes.c_int
_b = ctypes.c_bool


class SlamConfig(ctypes.Structure):
    """SlamConfig (slamtypes.h:142-250), 324 bytes."""
    _fields_ = [
        ("debug", _b),
        ("x0", _f), ("y0", _f), ("z0", _f), ("roll0", _f), ("pitch0", _f), ("yaw0", _f),
        ("vx0", _f), ("vy0", _f), ("vz0", _f), ("vroll0", _f), ("vpitch0", _f), ("vyaw0", _f),
        ("followTrajectory", _b),
        ("ax", _f), ("ay", _f), ("az", _f), ("aroll", _f), ("apitch", _f), ("ayaw", _f),
        ("dt", _f),
        ("minRange", _f), ("maxRange", _f), ("maxBearing", _f),
        ("stdRange", _f), ("stdBearing", _f),
        ("clutterRate", _f), ("clutterDensity", _f), ("pd", _f),
        ("stdVxMap", _f), ("stdVyMap", _f), ("stdAxMap", _f), ("stdAyMap", _f),
        ("covVxBirth", _f), ("covVyBirth", _f),
        ("ps", _f), ("tau", _f), ("beta", _f),
        ("particlesPerFeature", _i), ("imageWidth", _i), ("imageHeight", _i),
        ("stdU", _f), ("stdV", _f), ("disparityBirth", _f), ("stdDBirth", _f),
        ("fx", _f), ("fy", _f), ("u0", _f), ("v0", _f),
        ("n_particles", _i), ("nPredictParticles", _i), ("subdividePredict", _i),
        ("resampleThresh", _f), ("birthWeight", _f), ("birthNoiseFactor", _f),
        ("gateBirths", _b), ("gateMeasurements", _b),
        ("gateThreshold", _f), ("minExpectedFeatureWeight", _f), ("minSeparation", _f),
        ("maxFeatures", _i),
        ("minFeatureWeight", _f),
        ("particleWeighting", _i), ("daughterMixtureType", _i), ("nSamples", _i), ("maxCardinality", _i),
        ("filterType", _i), ("distanceMetric", _i), ("maxSteps", _i), ("featureModel", _i), ("motionType", _i),
        ("mapEstimate", _i), ("cphdDistType", _i),
        ("nu", _f),
        ("labeledMeasurements", _b),
        ("l", _f), ("h", _f), ("a", _f), ("b", _f), ("stdAlpha", _f), ("stdEncoder", _f),
        ("saveAllMaps", _b), ("savePrediction", _b),
    ]

    def update_clutter_density(self):
        """clutterDensity = clutterRate / (2 maxBearing maxRange) in float (main.cpp:1065-1066)."""
        f = np.float32
        self.clutterDensity = float(f(self.clutterRate) / (f(2) * f(self.maxBearing) * f(self.maxRange)))
        return self

    def copy(self):
        c = SlamConfig()
        ctypes.memmove(ctypes.addressof(c), ctypes.addressof(self), ctypes.sizeof(SlamConfig))
        return c


assert ctypes.sizeof(SlamConfig) == 324
assert SlamConfig.pd.offset == 112 and SlamConfig.n_particles.offset == 196
assert SlamConfig.labeledMeasurements.offset == 292 and SlamConfig.saveAllMaps.offset == 320


def csr_from_maps(maps):
    """list of GAUSSIAN2D arrays -> (flat array, offsets[n+1] int32)."""
    sizes = np.array([len(m) for m in maps], dtype=np.int64)
    offsets = np.zeros(len(maps) + 1, dtype=np.int32)
    offsets[1:] = np.cumsum(sizes)
    flat = np.concatenate(maps) if len(maps) and offsets[-1] > 0 else np.zeros(0, GAUSSIAN2D)
    return np.ascontiguousarray(flat, dtype=GAUSSIAN2D), offsets


def maps_from_csr(flat, offsets):
    return [flat[offsets[i]:offsets[i + 1]] for i in range(len(offsets) - 1)]
