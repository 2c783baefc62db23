"""crdtm — MI355X-native batch-merge engine for CRDTree (host-side package)."""
from .operation import Add, Batch, Delete  # noqa: F401
