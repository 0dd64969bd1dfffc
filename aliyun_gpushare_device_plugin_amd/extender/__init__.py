"""The gpushare scheduler extender (filter / bind over HTTP) for MI355X nodes."""
from .core import TP_GROUP_LABEL, TP_SIZE_LABEL, Extender, NodeState, serve_http  # noqa: F401
from .leader import LeaderElector  # noqa: F401
