"""``python -m paddle_hackathon_amd.distributed.fleet.launch`` (reference:
python/paddle/distributed/fleet/launch.py): the collective / parameter-server launcher."""
from ..spawn import launch

if __name__ == "__main__":
    import sys
    sys.exit(launch())
