"""Import-only stub for biopython's Bio.PDB (reference protein.py:24). Never called on the path."""


class PDBParser:  # pragma: no cover - stub
    def __init__(self, *a, **k):
        raise RuntimeError("Bio.PDB is not available in this container (oracle shim)")
