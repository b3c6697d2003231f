"""``fleet.elastic`` (reference: python/paddle/distributed/fleet/elastic): the elastic manager
(parallel/elastic.py; ``python -m paddle_hackathon_amd.distributed.fleet.elastic`` runs it)."""
from ...elastic import *  # noqa: F401,F403
from ...elastic import ElasticManager, ElasticStatus, ElasticLevel, enable_elastic, launch_elastic, main  # noqa: F401
