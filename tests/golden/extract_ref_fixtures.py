"""Extract the numeric data of the two pickled fixtures the reference ships
into tests/golden/ref_fixtures.npz -- WITHOUT unpickling them.

  /root/reference/uva_human_pp_video_act_model/normalizer.pkl  (a pickled LinearNormalizer:
      per field "action" / "agent_pos" / "image" a ParameterDict {offset, scale,
      input_stats {max, mean, min, std}}; every tensor's storage is a nested torch.save blob
      behind torch.storage._load_from_bytes, normalizer.py:195-297)
  /root/reference/prepared_data/language_latents.pkl  (dict cup / towel / mouse -> float32[512]
      numpy arrays through numpy.core.multiarray._reconstruct)

Nothing in either file is executed: the outer pickle is only READ as an opcode stream by
pickletools.genops (a disassembler: it constructs no object and resolves no global), keys are
taken from the string opcodes (with the pickle memo followed for repeated keys), and
  * each nested storage blob is loaded by torch.load(weights_only=True);
  * each numpy array is the raw little-endian float32 payload of its SHORT_BINBYTES/BINBYTES
    opcode (dtype '<f4' and the 512-element shape are checked against the opcode stream).
Run here (the reference exists only in this container); the .npz is the committed fixture.
"""
import io
import os
import pickletools
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_fixtures.npz")
STRING_OPS = {"SHORT_BINUNICODE", "BINUNICODE", "UNICODE", "BINUNICODE8"}
BYTES_OPS = {"SHORT_BINBYTES", "BINBYTES", "BINBYTES8"}
GET_OPS = {"BINGET", "LONG_BINGET", "GET"}


def string_stream(path):
    """-> [(kind, value)] in stream order: ("str", s) for every string pushed (directly or from the
    memo) and ("bytes", b) for every bytes payload.  Memo indices are counted for every MEMOIZE
    (PUT-style opcodes do not occur in these protocol-4 files: checked)."""
    data = open(path, "rb").read()
    memo, out, last = {}, [], None
    for op, arg, _ in pickletools.genops(data):
        name = op.name
        if name in ("PUT", "BINPUT", "LONG_BINPUT"):
            raise RuntimeError(f"{path}: unexpected {name}")
        if name == "MEMOIZE":
            memo[len(memo)] = last
        if name in STRING_OPS:
            last = ("str", arg)
            out.append(last)
        elif name in GET_OPS:
            last = memo.get(arg)
            if last is not None:
                out.append(last)
        elif name in BYTES_OPS:
            last = ("bytes", arg)
            out.append(last)
        else:
            last = None
    return out


def normalizer_params(path):
    """{"<field>/<offset|scale|input_stats/max|...>": float32 array}"""
    fields = ("action", "agent_pos", "image")
    res, field, stats = {}, None, False
    pending = None
    for kind, v in string_stream(path):
        if kind == "str":
            if v in fields:
                field, stats = v, False
            elif v == "input_stats":
                stats = True
            elif v in ("offset", "scale", "max", "mean", "min", "std"):
                pending = v
        elif kind == "bytes":
            st = torch.load(io.BytesIO(v), weights_only=True)  # nested legacy torch.save of one storage
            t = torch.tensor([], dtype=st.dtype).set_(st) if not torch.is_tensor(st) else st
            key = f"{field}/{'input_stats/' if stats else ''}{pending}"
            assert field is not None and pending is not None and key not in res, key
            res[key] = t.float().numpy().copy()
            pending = None
    return res


def language_latents(path):
    res, key = {}, None
    stream = string_stream(path)
    for i, (kind, v) in enumerate(stream):
        if kind == "str" and v in ("cup", "towel", "mouse"):
            key = v
        elif kind == "str" and v == "f4":
            assert stream[i + 1] == ("str", "<"), "expected a little-endian float32 dtype"
        elif kind == "bytes" and key is not None and len(v) > 1:  # (b"b" is _reconstruct's dtype char)
            assert len(v) == 512 * 4, (key, len(v))
            res[key] = np.frombuffer(v, dtype="<f4").copy()
            key = None
    assert sorted(res) == ["cup", "mouse", "towel"], sorted(res)
    return res


def main():
    norm = normalizer_params(os.path.join(REF, "uva_human_pp_video_act_model", "normalizer.pkl"))
    lat = language_latents(os.path.join(REF, "prepared_data", "language_latents.pkl"))
    out = {f"normalizer/{k}": v for k, v in norm.items()}
    out.update({f"language_latents/{k}": v for k, v in lat.items()})
    np.savez(OUT, **out)
    for k, v in out.items():
        print(f"{k:40s} {v.shape} {v[:4]}")
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
