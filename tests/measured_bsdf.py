"""Writes RGL-format measured BRDF tensor files (".bsdf", the layout pbrt's Tensor reader takes:
bxdfs.cpp:734-816) for the measured-material tests.  No measured data ships with the reference
or this image, so the tables are synthesised from an analytic microfacet model: a GGX normal
distribution (ndf), its projected area (sigma), the visible-normal density in the unit-square
parameterisation pbrt's MeasuredBxDF warps through (vndf), a smooth luminance warp and a
Fresnel-tinted spectral table (spectra).  The loader and the BxDF only need the structure;
the physical plausibility keeps the renders meaningful (finite, energy below 1)."""
import struct

import numpy as np


def _u2theta(u):
    return u * u * (np.pi / 2)


def _u2phi(u):
    return (2 * u - 1) * np.pi


def _ggx_d(cos_m, alpha):
    a2 = alpha * alpha
    return a2 / (np.pi * ((a2 - 1) * cos_m * cos_m + 1) ** 2)


def _sigma(cos_o, alpha):
    # projected microfacet area for GGX: cos_o * (1 + Lambda(wo)) (Smith)
    t2 = np.maximum(0.0, 1 - cos_o ** 2) / np.maximum(cos_o ** 2, 1e-12)
    lam = (-1 + np.sqrt(1 + alpha ** 2 * t2)) / 2
    return np.maximum(cos_o, 1e-4) * (1 + lam)


def write_tensor(path, fields):
    """fields: {name: ndarray (float32 or uint8)} -> the tensor_file layout"""
    dt_code = {np.dtype(np.uint8): 1, np.dtype(np.float32): 10}
    items = [(k, np.ascontiguousarray(v)) for k, v in fields.items()]
    header = b"tensor_file\0" + bytes([1, 0]) + struct.pack("<I", len(items))
    desc_len = sum(2 + len(k) + 2 + 1 + 8 + 8 * v.ndim for k, v in items)
    offset = len(header) + desc_len
    desc, blobs = b"", b""
    for k, v in items:
        offset_k = offset + len(blobs)
        desc += struct.pack("<H", len(k)) + k.encode() + struct.pack("<HBQ", v.ndim, dt_code[v.dtype], offset_k)
        desc += b"".join(struct.pack("<Q", s) for s in v.shape)
        blobs += v.tobytes()
    with open(path, "wb") as fp:
        fp.write(header + desc + blobs)


def make_bsdf(path, alpha=0.3, n_theta=6, n_phi=1, res=16, n_wl=8, tint=(0.95, 0.6, 0.3), jitter=0.0, seed=0,
              phi_range=(-np.pi, np.pi)):
    rng = np.random.default_rng(seed)
    u = np.linspace(0, 1, res, dtype=np.float64)
    ux, uy = np.meshgrid(u, u)  # [y][x]: x = theta coordinate, y = phi coordinate
    theta_m, phi_m = _u2theta(ux), _u2phi(uy)
    ndf = _ggx_d(np.cos(theta_m), alpha)
    sigma = _sigma(np.cos(_u2theta(ux)), alpha) * (1 + 0.05 * np.cos(_u2phi(uy)))
    theta_i = np.linspace(0, np.radians(80), n_theta)
    phi_i = np.array([0.0]) if n_phi == 1 else np.linspace(phi_range[0], phi_range[1], n_phi)
    wl = np.linspace(360, 830, n_wl)
    jac = 2 * np.pi ** 2 * np.maximum(ux, 1e-6) * np.sin(theta_m)
    vndf = np.zeros((len(phi_i), n_theta, res, res))
    lum = np.zeros_like(vndf)
    spectra = np.zeros((len(phi_i), n_theta, n_wl, res, res))
    fres = np.interp(wl, [360, 595, 830], tint)
    for a, po in enumerate(phi_i):
        for b, to in enumerate(theta_i):
            wo = np.array([np.sin(to) * np.cos(po), np.sin(to) * np.sin(po), np.cos(to)])
            pm = phi_m + (po if n_phi == 1 else 0)
            wm = np.stack([np.sin(theta_m) * np.cos(pm), np.sin(theta_m) * np.sin(pm), np.cos(theta_m)], -1)
            dots = np.maximum(wm @ wo, 0)
            vndf[a, b] = ndf * dots * jac + 1e-3
            lum[a, b] = 1 + 0.3 * ux * uy + 0.2 * np.cos(to) * ux
            g = 0.8 + 0.2 * dots
            for k in range(n_wl):
                spectra[a, b, k] = fres[k] * g * (1 + 0.1 * uy)
    if jitter:
        vndf *= 1 + jitter * rng.random(vndf.shape)
        spectra *= 1 + jitter * rng.random(spectra.shape)
    write_tensor(path, {
        "description": np.frombuffer(b"synthetic GGX", np.uint8),
        "theta_i": theta_i.astype(np.float32),
        "phi_i": phi_i.astype(np.float32),
        "ndf": ndf.astype(np.float32),
        "sigma": sigma.astype(np.float32),
        "vndf": vndf.astype(np.float32),
        "luminance": lum.astype(np.float32),
        "spectra": spectra.astype(np.float32),
        "wavelengths": wl.astype(np.float32),
        "jacobian": np.array([1], np.uint8),
    })
    return path
