"""``Problem.solveInverse`` (``source/jax_plate/Problem.py:641-914``).

Same arguments, optimizer names, scaling/relative-start semantics, report text
and ``.npz`` history log as the reference.  The loss is the fused GPU
forward + adjoint sweep; ``distributed=True`` shards the frequencies over the
ranks of an initialised ``torch.distributed`` group (one all-reduce per
evaluation, every rank runs the identical optimiser).  Extra optimizer:
``'lbfgs'`` (BASELINE.json C5).
"""
from __future__ import annotations

import os
from time import gmtime, perf_counter, strftime

import numpy as np
import torch
from scipy.optimize import OptimizeResult, differential_evolution, shgo

from . import Optimizers as opt
from .Input import Compressor

_LOCAL = {("trust_region", "tr"): opt.optimize_trust_region, ("coord_descent", "cd"): opt.optimize_cd,
          ("coord_descent_mem", "cd_mem"): opt.optimize_cd_mem2, ("grad_descent", "gd"): opt.optimize_gd,
          ("lbfgs", "l-bfgs"): opt.optimize_lbfgs}


def _a2s(s):
    return s if isinstance(s, str) else np.array2string(np.array(s), separator=', ', precision=5)


def solve_inverse(prob, arg0, loss_type: str, optimizer: str, compression=(False, 0), comp_alg: int = 1,
                  ref_fr=None, use_rel: bool = False, use_scaling: bool = False, use_constraints: bool = False,
                  report: bool = True, log: bool = True, case_name: str = '', uid: str = None,
                  extra_info: str = '', log_dir: str = None, distributed: bool = False, **opt_kwargs):
    if ref_fr is None:
        ref_fr = getattr(prob, 'reference_fr', None)
        if ref_fr is None:
            raise ValueError('Cannot solve inverse problem as `ref_fr` argument was not provided and the '
                             "Problem object doesn't have a reference_fr attribute.")
    ref_fr = [np.asarray(ref_fr[0]), np.asarray(ref_fr[1])]
    if not isinstance(compression, tuple):
        raise TypeError(f'`compression` argument should have a type `tuple`,not {type(compression)}.')
    if len(compression) != 2:
        raise ValueError(f'`compression` tuple should have 2 elements, not {len(compression)}.')
    if compression[0]:
        comp = Compressor(ref_fr[0], ref_fr[1], compression[1], comp_alg)
        ref_fr[0], ref_fr[1] = comp(compression[1])

    arg0 = np.array(arg0, dtype=np.float64)
    scaling = None
    if arg0.ndim == 1:
        if use_rel:
            if getattr(prob, 'parameters', None) is None:
                raise ValueError('Cannot use `arg0` as relative coefficients of correction as Problem object has '
                                 'no `parameters` attribute.')
            x0 = np.asarray(prob.parameters) * (arg0 + 1)
            if use_scaling:
                scaling, x0 = x0, arg0 + 1
        else:
            x0 = arg0
            if use_scaling:
                scaling, x0 = x0, np.ones_like(x0)
    elif arg0.ndim == 2:
        if use_scaling:
            scaling = np.max(np.abs(arg0), axis=1)
            x0 = arg0 / scaling[:, None]
        else:
            x0 = arg0
    else:
        raise ValueError('Invalid shape of `arg0` argument.')

    loss = prob.getLossFunction(ref_fr[0], ref_fr[1], loss_type, scaling, distributed=distributed)
    scale_arr = np.ones_like(x0) if scaling is None else (np.tile(scaling, (2, 1)).T if x0.ndim == 2 else scaling)

    local = next((fn for names, fn in _LOCAL.items() if optimizer in names), None)
    if local is not None:
        fn, call_x0 = local, x0
        if local is opt.optimize_trust_region and 'model' not in opt_kwargs and opt_kwargs.get('exact_hessian', True):
            # exact Hessian from one GPU sweep per model (factors reused per direction)
            opt_kwargs['model'] = prob.getLossHessianFunction(ref_fr[0], ref_fr[1], loss_type, scaling,
                                                              distributed=distributed)
        opt_kwargs.pop('exact_hessian', None)
    elif optimizer in ('de', 'shgo'):
        def np_loss(x):
            return float(loss(torch.as_tensor(np.asarray(x, dtype=np.float64))))
        vg = opt.value_and_grad(loss)
        if optimizer == 'de':
            fn = lambda f, bounds, **kw: differential_evolution(np_loss, bounds, **kw)   # noqa: E731
        else:
            if use_constraints:
                raise NotImplementedError('material constraints for shgo are not provided by this build')
            o = dict(opt_kwargs.pop('options', {}))
            o['jac'] = lambda x: vg(x)[1]
            fn = lambda f, bounds, **kw: shgo(np_loss, bounds, options=o, **kw)          # noqa: E731
        call_x0 = [tuple(b) for b in x0]
    else:
        raise ValueError(f'Optimizer type `{optimizer}` is not supported!')

    t0 = perf_counter()
    result = fn(loss, call_x0, **opt_kwargs)
    elapsed = (perf_counter() - t0) / 60

    if optimizer in ('de', 'shgo'):
        result = OptimizeResult(dict(result))
        result.f = result.fun
        result.x_history = [list(result.population)] if optimizer == 'de' else [list(getattr(result, 'xl', []))]
        result.f_history = [-1.0]
        result.status = result.message
        result.niter = result.nit
        result.grad_history = []
    if use_scaling:
        d = result._asdict() if hasattr(result, '_asdict') else dict(result)
        d['x'] = np.asarray(d['x']) * (scale_arr if scale_arr.ndim == 1 else scale_arr[:, 1])
        result = opt.optResult(**{k: d[k] for k in opt.optResult._fields}) if hasattr(result, '_asdict') \
            else OptimizeResult(d)

    full = case_name + (strftime("%d_%m_%Y_%H_%M_%S", gmtime()) if uid is None else uid)
    log_dir = log_dir or os.path.join(os.path.dirname(os.path.abspath(__file__)), 'optimization')
    rank0 = not (torch.distributed.is_available() and torch.distributed.is_initialized()) \
        or torch.distributed.get_rank() == 0
    if report and rank0:
        rel1 = rel2 = 'Unknown'
        if getattr(prob, 'parameters', None) is not None:
            p0 = np.asarray(prob.parameters)
            if arg0.ndim != 2:
                rel1 = (np.asarray(x0) * scale_arr - p0) / p0
            rel2 = (np.asarray(result.x) - p0) / p0
        comp_str = f'Using compression algorithm {comp_alg} with {compression[1]} points.\n' if compression[0] else ''
        kind = 'parameters' if arg0.ndim == 1 else 'bounds'
        rep = (f'{prob.accelerometer}\n{prob.material}\n{prob.geometry}\n' + extra_info + comp_str +
               f'Starting {kind}: {_a2s(np.asarray(x0) * scale_arr)}.\n'
               f'With relative error: {_a2s(rel1)}.\n'
               f'Initial loss: {result.f_history[0]}.\n'
               f'Elapsed time: {elapsed} min.\n'
               f'After optimization: {_a2s(result.x)}.\n'
               f'With relative error: {_a2s(rel2)}.\n'
               f'Resulting loss: {result.f}.\n'
               f'Optimization status: {result.status}.\n'
               f'Optimizer parameters: {opt_kwargs}.\n'
               f'Optimizer type: {optimizer}.\n'
               f'Scaling parameters used: {scale_arr}.\n')
        print(rep, end='')
        os.makedirs(log_dir, exist_ok=True)
        with open(os.path.join(log_dir, full + '.txt'), 'w+') as fh:
            fh.write(rep)
    if log and rank0:
        os.makedirs(log_dir, exist_ok=True)
        np.savez_compressed(os.path.join(log_dir, full), x=np.array(list(result.x_history) + [result.x]),
                            f=np.array(list(result.f_history) + [result.f]), k=np.array([result.niter]))
    return result
