"""``fleet.elastic.manager`` module path."""
from ...elastic import ElasticManager, ElasticStatus, ElasticLevel  # noqa: F401
