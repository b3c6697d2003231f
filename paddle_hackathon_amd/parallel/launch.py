"""``python -m paddle_hackathon_amd.distributed.launch`` entry point."""
import sys

from .spawn import launch

if __name__ == "__main__":
    sys.exit(launch())
