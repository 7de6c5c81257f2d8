"""A pickle reader that executes nothing: it walks a pickle's opcodes and
builds inert records, to read the reference's shipped committee weights
(models/pretrained/classifier_{gnb,sgd,xgb}.it_{0..4}.pkl, written by
joblib.dump at deam_classifier.py:331-333 and copied per user at
amg_test.py:347-351) as plain arrays.

Test infrastructure (tests/golden/gen_pretrained.py).  Untrusted input: no
GLOBAL is ever resolved or imported, no REDUCE is ever called.  A GLOBAL becomes
a Global(module, name) record, a REDUCE a Call(func, args) record, a NEWOBJ an
Obj(cls, args) record whose BUILD state is stored on it.  These shapes are
interpreted, by their (module, name) strings only:
  * numpy.dtype(str, ...) + BUILD state (.., byteorder, ..)  -> np.dtype
  * numpy.core.multiarray.scalar(dtype, bytes)              -> np.frombuffer
  * joblib.numpy_pickle.NumpyArrayWrapper + BUILD {shape, order, dtype, ...}:
    joblib writes the array's raw bytes into the stream right after that
    BUILD (numpy_pickle.py NumpyArrayWrapper.write_array; a padding-length
    byte first when the wrapper records an alignment) -> np.ndarray
  * numpy.core.multiarray._reconstruct(ndarray, ...) + BUILD (version, shape,
    dtype, fortran, raw bytes)                                -> np.ndarray
  * builtins.bytearray(bytes)                                -> bytes
Anything else stays a record; an opcode outside the supported subset raises.
"""
from __future__ import annotations

import io
import pickletools

import numpy as np


class Global:
    def __init__(self, module, name):
        self.module, self.name = module, name

    def __repr__(self):
        return f"Global({self.module}.{self.name})"

    def is_(self, module, name):
        return self.module == module and self.name == name


class Call:
    def __init__(self, func, args):
        self.func, self.args, self.state = func, args, None

    def __repr__(self):
        return f"Call({self.func!r}, {self.args!r})"


class Obj:
    def __init__(self, cls, args):
        self.cls, self.args, self.state = cls, args, None

    def __repr__(self):
        return f"Obj({self.cls!r})"


_MARK = object()


def _is_global(x, module, name):
    return isinstance(x, Global) and x.is_(module, name)


def _dtype(d):
    if isinstance(d, np.dtype):
        return d
    raise ValueError(f"not a dtype: {d!r}")


def walk(data: bytes):
    """The object a pickle describes, with every non-interpreted object an
    inert record (see the module docstring)."""
    f = io.BytesIO(data)
    stack, memo = [], {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    while True:
        code = f.read(1)
        if not code:
            raise ValueError("pickle ended without STOP")
        op = pickletools.code2op.get(code.decode("latin-1"))
        if op is None:
            raise ValueError(f"unknown opcode {code!r} at {f.tell() - 1}")
        arg = op.arg.reader(f) if op.arg is not None else None
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            return stack.pop()
        if n == "GLOBAL":
            mod, name = arg.split(" ", 1)
            stack.append(Global(mod, name))
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            stack.append(Global(mod, name))
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n == "MARK":
            stack.append(_MARK)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "DICT":
            items = pop_mark()
            stack.append(dict(zip(items[0::2], items[1::2])))
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "LIST":
            stack.append(pop_mark())
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            for k, v in zip(items[0::2], items[1::2]):
                stack[-1][k] = v
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()  # (before reading stack[-1]: the list sits below the mark)
            stack[-1].extend(items)
        elif n in ("BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8", "UNICODE", "BINSTRING", "SHORT_BINSTRING",
                   "STRING"):
            stack.append(arg)
        elif n in ("BINBYTES", "SHORT_BINBYTES", "BINBYTES8", "BYTEARRAY8"):
            stack.append(bytes(arg))
        elif n in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG"):
            stack.append(arg)
        elif n in ("BINFLOAT", "FLOAT"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n in ("NEWOBJ", "NEWOBJ_EX"):
            if n == "NEWOBJ_EX":
                stack.pop()  # kwargs
            args = stack.pop()
            cls = stack.pop()
            stack.append(Obj(cls, args))
        elif n == "REDUCE":
            args = stack.pop()
            func = stack.pop()
            if _is_global(func, "numpy", "dtype") and isinstance(args[0], str):
                stack.append(np.dtype(args[0]))
            elif _is_global(func, "numpy.core.multiarray", "scalar"):
                stack.append(np.frombuffer(args[1], dtype=_dtype(args[0]))[0])
            elif _is_global(func, "builtins", "bytearray"):
                stack.append(bytes(args[0]) if args else b"")
            else:
                stack.append(Call(func, args))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, np.dtype):
                # numpy's dtype state: (version, byteorder, subarray, names, fields, elsize, alignment, flags)
                bo = state[1] if isinstance(state, tuple) and len(state) > 1 else "|"
                stack[-1] = obj.newbyteorder(bo) if bo in "<>" else obj
            elif isinstance(obj, Obj) and _is_global(obj.cls, "joblib.numpy_pickle", "NumpyArrayWrapper"):
                stack[-1] = _read_joblib_array(f, state)
            elif isinstance(obj, Call) and _is_global(obj.func, "numpy.core.multiarray", "_reconstruct"):
                _, shape, dt, fortran, raw = state
                a = np.frombuffer(raw, dtype=_dtype(dt))
                stack[-1] = a.reshape(shape, order="F" if fortran else "C").copy()
            elif isinstance(obj, (Obj, Call)):
                obj.state = state
            else:
                raise ValueError(f"BUILD on {type(obj).__name__}")
        else:
            raise ValueError(f"unsupported opcode {n}")


def _read_joblib_array(f, st):
    """The raw array joblib wrote after a NumpyArrayWrapper's BUILD."""
    if not isinstance(st, dict) or not isinstance(st.get("dtype"), np.dtype):
        raise ValueError("NumpyArrayWrapper without a dtype")
    dt, shape, order = st["dtype"], tuple(st["shape"]), st.get("order", "C")
    if dt.hasobject:
        raise ValueError("object arrays are not read (they would be a nested pickle)")
    if st.get("numpy_array_alignment_bytes") is not None:
        pad = f.read(1)[0]
        f.read(pad)
    count = int(np.prod(shape, dtype=np.int64)) if shape else 1
    raw = f.read(count * dt.itemsize)
    if len(raw) != count * dt.itemsize:
        raise ValueError("truncated array data")
    return np.frombuffer(raw, dtype=dt).reshape(shape, order="F" if order == "F" else "C").copy()


def state_of(obj):
    """An Obj's (or Call's) BUILD state dict."""
    if not isinstance(obj, (Obj, Call)) or not isinstance(obj.state, dict):
        raise ValueError(f"{obj!r} carries no state dict")
    return obj.state


def read_gnb(data):
    """sklearn 0.24.1 GaussianNB: theta_, sigma_ (the variance incl. epsilon_), class_prior_, classes_."""
    o = walk(data)
    if not _is_global(o.cls, "sklearn.naive_bayes", "GaussianNB"):
        raise ValueError(f"not a GaussianNB: {o!r}")
    s = state_of(o)
    var = s["sigma_"] if "sigma_" in s else s["var_"]
    return {"theta": s["theta_"], "var": var, "class_prior": s["class_prior_"], "classes": s["classes_"],
            "epsilon": float(s["epsilon_"])}


def read_sgd(data):
    """sklearn 0.24.1 SGDClassifier: coef_, intercept_, classes_, loss."""
    o = walk(data)
    if not _is_global(o.cls, "sklearn.linear_model._stochastic_gradient", "SGDClassifier"):
        raise ValueError(f"not an SGDClassifier: {o!r}")
    s = state_of(o)
    return {"coef": s["coef_"], "intercept": s["intercept_"], "classes": s["classes_"], "loss": s["loss"]}


def read_xgb(data):
    """xgboost 1.3.3 XGBClassifier: the booster's serialised JSON ('Model' part:
    the save_model schema ce_amd.xgb.XgbForest.from_json reads), n_classes_."""
    import json

    o = walk(data)
    if not _is_global(o.cls, "xgboost.sklearn", "XGBClassifier"):
        raise ValueError(f"not an XGBClassifier: {o!r}")
    s = state_of(o)
    b = s["_Booster"]
    if not (isinstance(b, Obj) and _is_global(b.cls, "xgboost.core", "Booster")):
        raise ValueError(f"_Booster is {b!r}")
    handle = state_of(b)["handle"]
    doc = json.loads(bytes(handle).decode("utf-8"))
    return {"model": doc["Model"], "config": doc.get("Config"), "n_classes": int(s["n_classes_"]),
            "objective": s.get("objective")}
