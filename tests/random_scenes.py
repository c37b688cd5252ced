"""Seeded adversarial scenes for the proof-based skips (test helper).

The kernel skips work by proofs that rest on host-derived error bounds: the
f64 primary-ray cone cull, the FMA secondary-ray prefilter, the cluster walk
and its behind-origin rule.  The built-in scenes exercise them
only in one regime, so this generator builds scenes that stress the slack:
- sphere counts from 1 to 1,060 (265 groups; the four-wave kernels' LDS image holds up to 164);
- radii log-uniform over 1e-3 ... 1e2 of a world scale itself drawn from
  1e-2 ... 1e2 (so the reference's absolute eps = 1e-4 is met at every scale),
  or, in "cloud" scenes, within one decade (the scene-wide prefilter bound
  then pays, and the cluster walk runs);
- overlapping, nested, near-coincident and near-tangent sphere pairs;
- four cameras per scene: outside the cloud, inside a sphere, on a sphere's
  surface, and one with spheres placed tangent to film rays (grazing hits);
- random materials: diffuse, specular, dielectric (IOR < 1 and > 1), emissive,
  with and without the sky term.
Scenes are rt_scalar_sphere records (main.cpp:17-21) converted to groups as
ConvertScalarSpheresToSIMDSpheres does (rt.scene_from_spheres)."""
import numpy as np

F = np.float32


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def _camera_pos(look, distance, x_angle, y_height):
    return np.array([np.cos(x_angle) * distance + look[0], y_height + look[1], np.sin(x_angle) * distance + look[2]])


def make(seed: int, n_max: int = 1060):
    """Returns dict(spheres (N,20) f32, use_sky, cameras=[(look_at, distance, x_angle, y_height, kind)])."""
    rng = np.random.default_rng(seed)
    scale = float(10.0 ** rng.uniform(-2, 2))
    # "cloud" scenes (radii within one decade, like the built-in Floating Spheres)
    # keep the scene-wide prefilter bound useful, so the cluster walk and its
    # behind-origin rule run; "wide" scenes (radii over three decades, a huge
    # sphere) take the per-lane thresholds
    cloud = rng.random() < 0.4
    if cloud:
        n = int(rng.integers(8, 257))
    else:  # mostly small scenes (fast oracle), some large, one in ten at the maximum
        n = int(rng.choice([rng.integers(1, 9), rng.integers(9, 80), rng.integers(80, 300), n_max],
                           p=[0.25, 0.45, 0.2, 0.1]))
    extent = scale * rng.uniform(1.0, 4.0)
    c = rng.uniform(-extent, extent, (n, 3))
    r = scale * (10.0 ** rng.uniform(np.log10(0.05), np.log10(0.3), n) if cloud else 10.0 ** rng.uniform(-3, 0, n))
    if not cloud and n > 4 and rng.random() < 0.3:  # one huge sphere (a ground, or a sphere around everything)
        k = rng.integers(n)
        r[k] = scale * 10.0 ** rng.uniform(1, 2)
        if rng.random() < 0.5:
            c[k] = [0.0, -r[k] - scale * 0.5, 0.0]
    # adversarial pairs: tangent (outside / inside), near-coincident, nested
    for i in range(1, n):
        u = rng.random()
        if u < 0.12:
            d = _unit(rng.normal(size=3))
            c[i] = c[i - 1] + d * (r[i - 1] + r[i]) * (1.0 + rng.uniform(-1e-6, 1e-6))
        elif u < 0.18:
            d = _unit(rng.normal(size=3))
            big, small = max(r[i - 1], r[i]), min(r[i - 1], r[i])
            r[i - 1], r[i] = big, small
            c[i] = c[i - 1] + d * (big - small) * (1.0 - rng.uniform(0, 1e-6))
        elif u < 0.22:
            c[i] = c[i - 1] * (1.0 + rng.uniform(-1e-7, 1e-7, 3))
            r[i] = r[i - 1] * (1.0 + rng.uniform(-1e-7, 1e-7))
        elif u < 0.26:
            c[i] = c[i - 1] + rng.uniform(-0.5, 0.5, 3) * r[i - 1]
    sp = np.zeros((n, 20), F)
    sp[:, 0:3] = c
    sp[:, 4] = r
    for i in range(n):
        m = sp[i, 8:20]  # Color(4) Emissive(4) Specular IOR pad pad
        m[0:3] = rng.uniform(0.05, 1.0, 3)
        kind = rng.random()
        if kind < 0.15:
            m[9] = rng.choice([1.5, 1.33, 2.4, 1.0 / 1.5])
        elif kind < 0.4:
            m[8] = rng.uniform(0.0, 1.0)
        if rng.random() < 0.1:
            m[4:7] = rng.uniform(0.0, 4.0, 3)
    use_sky = bool(rng.random() < 0.5)
    centroid = c.mean(0)
    cams = [(centroid, float(extent * rng.uniform(2.0, 4.0)), float(rng.uniform(-6, 6)),
             float(extent * rng.uniform(-0.5, 0.5)), "outside")]
    k = int(np.argmax(r))
    cams.append((c[k], float(r[k] * rng.uniform(0.1, 0.8)), float(rng.uniform(-6, 6)), 0.0, "inside"))
    k = rng.integers(n)
    ang = float(rng.uniform(-6, 6))
    cams.append((c[k], float(np.float32(r[k])), ang, 0.0, "on_surface"))
    cams.append((centroid, float(extent * rng.uniform(1.5, 3.0)), float(rng.uniform(-6, 6)),
                 float(extent * rng.uniform(-0.3, 0.3)), "grazing"))
    return {"spheres": sp, "use_sky": use_sky, "cameras": cams, "scale": scale, "n": n, "cloud": cloud}


def add_grazing_spheres(rt, spec, W, H, count=4, seed=0):
    """Spheres tangent to film rays of the 'grazing' camera (distance from the
    pixel-centre ray = r (1 +- 1e-6)): returns a new spheres array."""
    rng = np.random.default_rng(seed)
    look, dist, ang, yh, _ = spec["cameras"][3]
    tmp = rt.scene_from_spheres(spec["spheres"], look_at=tuple(look), distance=dist, x_angle=ang, y_height=yh)
    cam = rt.camera_setup(tmp, W, H)
    v = lambda a: np.array([a.x, a.y, a.z], np.float64)
    cp, cx, cy, fc = v(cam.CameraPosition), v(cam.CameraX), v(cam.CameraY), v(cam.FilmCenter)
    extra = []
    for _ in range(count):
        x, y = rng.uniform(0, W), rng.uniform(0, H)
        ka = (-1.0 + 2.0 * x / W) * cam.FilmW * 0.5
        kb = (-1.0 + 2.0 * y / H) * cam.FilmH * 0.5
        d = _unit(fc - cp + ka * cx + kb * cy)
        t = spec["scale"] * rng.uniform(0.5, 3.0)
        rad = spec["scale"] * 10.0 ** rng.uniform(-2, -0.5)
        nrm = _unit(np.cross(d, rng.normal(size=3)))
        row = np.zeros(20, F)
        row[0:3] = cp + d * t + nrm * rad * (1.0 + rng.uniform(-1e-6, 1e-6))
        row[4] = rad
        row[8:11] = rng.uniform(0.1, 1.0, 3)
        extra.append(row)
    return np.concatenate([spec["spheres"], np.array(extra, F)])[: 4 * 265]


def build(rt, orc, spheres, use_sky, look, distance, x_angle, y_height):
    """(rt scene, oracle scene) sharing one sphere array and look-at point."""
    s = rt.scene_from_spheres(spheres, look_at=tuple(float(v) for v in look), use_sky=use_sky, distance=distance,
                              x_angle=x_angle, y_height=y_height)
    sp, groups, mats = rt.scene_arrays(s)
    o = orc.Scene(sp, groups, mats, look_at=tuple(float(v) for v in look), use_sky=use_sky, distance=distance,
                  x_angle=x_angle, y_height=y_height)
    return s, o
