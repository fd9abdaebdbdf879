"""Test-only stand-in for dm-tree's `map_structure` (recursive map over nested containers)."""


def map_structure(fn, *structs):
    s0 = structs[0]
    if isinstance(s0, (list, tuple)):
        out = [map_structure(fn, *xs) for xs in zip(*structs)]
        return type(s0)(out) if isinstance(s0, tuple) else out
    if isinstance(s0, dict):
        return {k: map_structure(fn, *[s[k] for s in structs]) for k in s0}
    return fn(*structs)
