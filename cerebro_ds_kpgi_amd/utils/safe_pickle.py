"""Restricted unpickling for the CTQ-format run records.

``models_info.pkl`` / ``jobs_info.pkl`` (the reference's CTQ record layout,
written by ``runtime.checkpoint.dump_infos``) hold only containers of
strings, numbers and booleans.  They are read back by resume and by the log
analytics, which may be pointed at any logs directory, so loading goes
through an unpickler that resolves no global except plain builtin containers
and numpy scalars: a pickle that names anything else (e.g. ``os.system``)
raises ``pickle.UnpicklingError`` instead of executing it.
"""

import io
import pickle

_ALLOWED = {
    ("builtins", "dict"), ("builtins", "list"), ("builtins", "tuple"), ("builtins", "set"),
    ("builtins", "frozenset"), ("builtins", "str"), ("builtins", "int"), ("builtins", "float"),
    ("builtins", "bool"), ("builtins", "complex"), ("builtins", "bytes"),
    ("collections", "OrderedDict"), ("collections", "defaultdict"),
    ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
}


class _Restricted(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super(_Restricted, self).find_class(module, name)
        raise pickle.UnpicklingError("refusing to load global {}.{}".format(module, name))


def load(f):
    """``pickle.load`` restricted to plain data (see module docstring)."""
    return _Restricted(f).load()


def loads(b):
    return _Restricted(io.BytesIO(b)).load()
