"""ctypes access to tools/libaero_mathhost.so (host build of aero_math.h)."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.environ.get('AERO_MATHHOST_SO') or os.path.join(ROOT, 'tools', 'libaero_mathhost.so')
FN = {'hypot': 0, 'atan2': 1, 'tanh': 2, 'sin': 3, 'cos': 4, 'log10': 5, 'sqrt': 6, 'fmod360': 7, 'div': 8,
      'sincos_s': 9, 'sincos_c': 10, 'log': 12, 'glibc_sin': 13, 'glibc_cos': 14}
_lib = None


def lib():
    global _lib
    if _lib is None:
        import sys
        sys.path.insert(0, os.path.join(ROOT, 'aero-cli_amd'))
        import build
        if not os.environ.get('AERO_MATHHOST_SO'):
            build.build_mathhost()
        _lib = ctypes.CDLL(SO)
        for f in ('aero_math_host_eval', 'aero_math_glibc_eval'):
            getattr(_lib, f).argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_size_t]
    return _lib


def _eval(f, fn, x, y):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.zeros_like(x) if y is None else np.ascontiguousarray(y, dtype=np.float64)
    out = np.empty_like(x)
    f(FN[fn], x.ctypes.data, y.ctypes.data, out.ctypes.data, x.size)
    return out


def evaluate(fn, x, y=None):
    return _eval(lib().aero_math_host_eval, fn, x, y)


def glibc(fn, x, y=None):
    return _eval(lib().aero_math_glibc_eval, fn, x, y)
