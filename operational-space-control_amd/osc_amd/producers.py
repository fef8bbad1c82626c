"""Host wrappers of the batched input producers (include/osc_producers.h):
the example drivers' per-tick target and contact-mask logic on the device, so a control step
(kinematics -> targets / mask -> solve) stays on the GPU.  Device tensors in, device tensors out,
launched on the current torch stream; no CPU fallback."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream, device):
    return (torch.cuda.current_stream(device) if stream is None else stream).cuda_stream


def tumbling_params(**overrides) -> _lib.OscTumblingParams:
    """osc_tumbling_params_default (the example's gains and joint addresses), then overrides."""
    p = _lib.OscTumblingParams()
    _lib.lib().osc_tumbling_params_default(ctypes.byref(p))
    for k, v in overrides.items():
        if k == "shin_qadr":
            p.shin_qadr[:] = list(v)
        else:
            setattr(p, k, float(v))
    return p


def tumbling_targets_into(out, qpos, qvel, site_xpos, t, t0, init_qpos, init_site_xpos,
                          params: _lib.OscTumblingParams | None = None, stream=None):
    """osc_tumbling_targets: examples/walter_sr_true_tumbling_mjjoint.cc:622-1019 for every env.
    out (nenv, 17, 6); qpos / init_qpos (nenv, nq); qvel (nenv, nv); site_xpos / init_site_xpos
    (nenv, 17, 3); t / t0 (nenv,)."""
    nenv, nq = qpos.shape
    nv = qvel.shape[1]
    ns = site_xpos.shape[1]
    params = params or tumbling_params()
    rc = _lib.lib().osc_tumbling_targets(nenv, ns, nq, nv, _p(qpos), _p(qvel), _p(site_xpos),
                                         _p(t), _p(t0), _p(init_qpos), _p(init_site_xpos),
                                         ctypes.byref(params), _p(out),
                                         ctypes.c_void_p(_stream(stream, qpos.device)))
    if rc != 0:
        raise _lib.OSCError("osc_tumbling_targets", rc)
    return out


def contact_geom_table(geom_bodyid, site_bodyid, ids) -> np.ndarray:
    """osc_contact_geom_table (host): the example's geom -> contact-site rule."""
    g = np.ascontiguousarray(geom_bodyid, dtype=np.int32)
    s = np.ascontiguousarray(site_bodyid, dtype=np.int32)
    i = np.ascontiguousarray(ids, dtype=np.int32)
    out = np.empty(len(g), dtype=np.int32)
    ptr = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    rc = _lib.lib().osc_contact_geom_table(len(g), ptr(g), len(s), ptr(s), len(i), ptr(i), ptr(out))
    if rc != 0:
        raise _lib.OSCError("osc_contact_geom_table", rc)
    return out


def contact_mask_into(out, ncon, geom_pairs, geom_to_site, stream=None):
    """osc_contact_mask_from_contacts: out (nenv, nc) float64; ncon (nenv,) int32; geom_pairs
    (nenv, max_con, 2) int32; geom_to_site (ngeom,) int32 (all device tensors)."""
    nenv, nc = out.shape
    max_con = geom_pairs.shape[1]
    rc = _lib.lib().osc_contact_mask_from_contacts(nenv, nc, max_con, _p(ncon), _p(geom_pairs),
                                                   geom_to_site.shape[0], _p(geom_to_site),
                                                   _p(out), ctypes.c_void_p(_stream(stream, out.device)))
    if rc != 0:
        raise _lib.OSCError("osc_contact_mask_from_contacts", rc)
    return out
