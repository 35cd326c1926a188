"""Counter-hash parameter initialisation shared by the golden generator and the tests.

Every parameter value is a pure function of (parameter name, flat index):
    seed  = fnv1a64(name)
    bits  = splitmix64(seed + index)
    u     = 2 * (bits >> 11) * 2**-53 - 1            in [-1, 1)
    value = u * scale(name, shape) + offset(name, shape)

so no weights are committed and the reference model (fixture generation) and
this build's oracle / HIP path (tests) load bit-identical fp32 weights.
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_pm1(name: str, n: int) -> np.ndarray:
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        bits = splitmix64(idx + np.uint64(fnv1a64(name)))
    u = (bits >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return (2.0 * u - 1.0)


def param_value(name: str, shape) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform_pm1(name, n)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "weight" and len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        v = u * np.sqrt(1.0 / fan_in)
    elif leaf == "weight":  # LayerNorm / GroupNorm affine
        v = 1.0 + 0.1 * u
    elif leaf == "bias":
        v = 0.05 * u
    else:  # embeddings, fake latents
        v = 0.05 * u
    return v.astype(np.float32).reshape(shape)


def hash_init_(module, prefix: str = ""):
    """Overwrite every parameter of a torch module in place (names relative to module)."""
    import torch
    with torch.no_grad():
        for name, p in module.named_parameters():
            p.copy_(torch.from_numpy(param_value(prefix + name, p.shape)))
    return module


def hash_tensor(name: str, shape, scale=1.0) -> np.ndarray:
    """Deterministic input tensor: uniform [-scale, scale)."""
    n = int(np.prod(shape))
    return (uniform_pm1(name, n) * scale).astype(np.float32).reshape(shape)


def hash_normal(name: str, shape) -> np.ndarray:
    """Deterministic ~N(0,1) tensor by Box-Muller on two hashed uniform streams."""
    n = int(np.prod(shape))
    u1 = (uniform_pm1(name + "#a", n) + 1.0) * 0.5
    u2 = (uniform_pm1(name + "#b", n) + 1.0) * 0.5
    u1 = np.clip(u1, 1e-12, 1.0)
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    return z.astype(np.float32).reshape(shape)
