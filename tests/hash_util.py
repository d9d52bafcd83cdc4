"""Shared setup of the SurfaceHash (useHash) tests (test infrastructure)."""
import math

import eslam_abi as A
import synthetic as S

# feet of a robot standing across a slope: the lowest points give a rare slope bucket,
# so sampleFromHash's relevance passes 0.8 and particles are replaced
SLOPE_FEET = [(0.25, 0.0, -0.18), (-0.25, 0.0, -0.18), (0.25, -0.5, -0.38), (-0.25, -0.5, -0.38)]


def hash_config(n, steps=8, bins=20, period=2, percentage=0.05):
    cfg = A.default_config()
    cfg.particle_count = n
    cfg.min_effective = n // 2
    cfg.measurement_threshold_distance = -1.0
    cfg.measurement_threshold_angle = -1.0
    cfg.hash_use = 1
    cfg.hash_period = period
    cfg.hash_percentage = percentage
    cfg.hash_angular_steps = steps
    cfg.hash_slope_bins = bins
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    return cfg


def hash_grid(cells=60):
    return S.rough_map(cells=cells, seed=11)


def rotated_grid(cells=60, yaw=0.3, tx=0.7, ty=-0.4):
    """A rough map whose grid frame is rotated/translated against the world (global2local)."""
    g = S.rough_map(cells=cells, seed=11)
    c, s = math.cos(yaw), math.sin(yaw)
    # global2local = inverse of grid2world [R | t]: [R^T | -R^T t]
    g.g2l = [c, s, 0.0, -(c * tx + s * ty), -s, c, 0.0, -(-s * tx + c * ty), 0.0, 0.0, 1.0, 0.0]
    return g


def slope_stream(steps):
    return S.step_stream(steps, feet=SLOPE_FEET, tilt=True)
