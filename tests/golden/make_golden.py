"""Generate golden vectors for the oracle from the reference's own Python models.

Runs ONLY in the build container (where /root/reference exists). The outputs
are plain JSON/NPZ data under tests/golden/; nothing from the reference's source
is copied. The reference's Python models are imported read-only from
/root/reference/python:

  * RangeBearingMeasurementModel.compute_measurement  (python/RangeBearingMeasurementModel.py:22-31)
  * RangeBearingMeasurementModel.invert_measurement   (python/RangeBearingMeasurementModel.py:67-73)
  * AckermanMotionModel.compute_motion                (python/AckermanMotionModel.py:23-40)
  * wrap_angle                                        (python/RangeBearingMeasurementModel.py:5-9)
  * ConstantVelocityMotionModel.compute_motion        (python/ConstantVelocityMotionModel.py:13-29; the
    module omits its numpy imports, so cos / sin / vstack are injected into
    its namespace before the call)

It also converts the reference's config-1 input data (python/controls_synth.txt,
python/measurements_synth.txt — data, not code) into a compact .npz fixture, and
the first steps of the reference's constant-velocity dataset
(matlab/measurements_synth_cv.txt) into config3_cv_data.npz.

Usage:  python3 -B tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

REF_PY = "/root/reference/python"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, REF_PY)
    import AckermanMotionModel as amm  # noqa: E402
    import ConstantVelocityMotionModel as cvm  # noqa: E402
    import RangeBearingMeasurementModel as rbm  # noqa: E402
    cvm.cos, cvm.sin, cvm.vstack = np.cos, np.sin, np.vstack  # the module's missing imports

    rng = np.random.RandomState(20261015)
    out = {"source": "reference python models (see make_golden.py header)"}

    # Ackerman: parameters from cfg/config.cfg (l, h, a, b)
    params = {"l": 1.415, "h": 0.38, "a": 1.89, "b": 0.5,
              "std_encoder": 1.0, "std_alpha": 0.034907}
    model = amm.AckermanMotionModel(params)
    cases = []
    poses = [(0.0, 0.0, 0.0)] + [tuple(v) for v in
                                 np.column_stack([rng.uniform(-20, 20, 63),
                                                  rng.uniform(-20, 20, 63),
                                                  rng.uniform(-3.1, 3.1, 63)])]
    for k, pose in enumerate(poses):
        if k == 0:
            v, alpha, dt = 2.77796, -0.186915, 0.1
        else:
            v, alpha, dt = rng.uniform(-3, 3), rng.uniform(-0.4, 0.4), rng.choice([0.1, 0.05, 0.2])
        newp = model.compute_motion(np.array(pose, dtype=float), v, alpha, dt).ravel()
        cases.append({"pose": list(pose), "v_encoder": float(v), "alpha": float(alpha),
                      "dt": float(dt), "out": [float(x) for x in newp]})
    out["ackerman"] = {"params": params, "cases": cases}

    # constant velocity (noise-free part): pose (x, y, z, yaw, vx, vy, vz, vyaw), planar (z = vz = 0)
    cv = cvm.ConstantVelocityMotionModel({"std_x": 0.5, "std_y": 0.0, "std_z": 0.0, "std_yaw": 0.0087,
                                          "std_pitch": 0.0})
    cvcases = []
    for _ in range(64):
        x, y, yaw = rng.uniform(-20, 20), rng.uniform(-20, 20), rng.uniform(-3.1, 3.1)
        vx, vy, vyaw = rng.uniform(-3, 3), rng.uniform(-1, 1), rng.uniform(-0.5, 0.5)
        dt = float(rng.choice([0.1, 0.05, 0.2]))
        newp = cv.compute_motion(np.array([x, y, 0.0, yaw, vx, vy, 0.0, vyaw]), dt).ravel()
        cvcases.append({"pose": [x, y, yaw, vx, vy, vyaw], "dt": dt,
                        "out": [float(newp[k]) for k in (0, 1, 3, 4, 5, 7)]})
    out["cv"] = {"cases": cvcases}

    # Range-bearing measurement model: h and h^-1
    sparams = {"max_range": 50.0, "max_bearing": float(np.pi), "std_range": 0.25,
               "std_bearing": 0.008727, "pd": 0.95, "clutter_rate": 20.0}
    mm = rbm.RangeBearingMeasurementModel(sparams)
    hcases = []
    pose0 = np.array([0.0, 0.0, 0.0])
    z = mm.compute_measurement(pose0, np.array([[3.0], [4.0]]))
    hcases.append({"pose": [0.0, 0.0, 0.0], "feature": [3.0, 4.0], "z": z[:, 0].tolist()})
    for _ in range(63):
        pose = np.array([rng.uniform(-10, 10), rng.uniform(-10, 10), rng.uniform(-3.1, 3.1)])
        feat = pose[:2] + rng.uniform(-30, 30, 2)
        z = mm.compute_measurement(pose, feat.reshape(2, 1))
        if z.shape[1] == 0:
            continue
        hcases.append({"pose": pose.tolist(), "feature": feat.tolist(), "z": z[:, 0].tolist()})
    out["measurement_h"] = {"params": sparams, "cases": hcases}

    icases = []
    for _ in range(64):
        pose = np.array([rng.uniform(-10, 10), rng.uniform(-10, 10), rng.uniform(-3.1, 3.1)])
        zz = np.array([[rng.uniform(0.5, 50.0)], [rng.uniform(-np.pi, np.pi)]])
        f = mm.invert_measurement(pose, zz)
        icases.append({"pose": pose.tolist(), "z": zz[:, 0].tolist(), "feature": f[:, 0].tolist()})
    out["measurement_hinv"] = {"cases": icases}

    angles = np.concatenate([rng.uniform(-20, 20, 60), [np.pi - 1e-3, -np.pi + 1e-3, 7.0, -7.0]])
    out["wrap_angle"] = {"in": angles.tolist(), "out": rbm.wrap_angle(angles.copy()).tolist()}

    with open(os.path.join(HERE, "models_golden.json"), "w") as f:
        json.dump(out, f, indent=1)

    # Config-1 data fixture: controls ("v, alpha" per line, comma separated, no header) and
    # measurements (range/bearing pairs per line, no header) -> ragged arrays.
    controls = []
    with open(os.path.join(REF_PY, "controls_synth.txt")) as f:
        for line in f:
            line = line.strip()
            if line:
                controls.append([float(x) for x in line.replace(",", " ").split()])
    meas_flat, meas_off = [], [0]
    with open(os.path.join(REF_PY, "measurements_synth.txt")) as f:
        for line in f:
            vals = [float(x) for x in line.split()]
            meas_flat.extend(vals)
            meas_off.append(len(meas_flat) // 2)
    np.savez_compressed(os.path.join(HERE, "config1_data.npz"),
                        controls=np.array(controls, dtype=np.float32),
                        meas=np.array(meas_flat, dtype=np.float32).reshape(-1, 2),
                        meas_offsets=np.array(meas_off, dtype=np.int64))
    # the reference's CV dataset (matlab/measurements_synth_cv.txt): '%' header, then
    # one step per line of range/bearing pairs; the first 40 steps
    cv_flat, cv_off = [], [0]
    with open(os.path.join(os.path.dirname(REF_PY), "matlab", "measurements_synth_cv.txt")) as f:
        for line in f:
            if line.startswith("%"):
                continue
            vals = [float(x) for x in line.split()]
            cv_flat.extend(vals)
            cv_off.append(len(cv_flat) // 2)
            if len(cv_off) > 40:
                break
    np.savez_compressed(os.path.join(HERE, "config3_cv_data.npz"),
                        meas=np.array(cv_flat, dtype=np.float32).reshape(-1, 2),
                        meas_offsets=np.array(cv_off, dtype=np.int64))
    print("wrote", len(cases), "ackerman,", len(cvcases), "cv,", len(hcases), "h,", len(icases), "hinv cases;",
          len(controls), "controls,", len(meas_off) - 1, "measurement steps")


if __name__ == "__main__":
    main()
