"""``paddle.distributed.cloud_utils`` (reference: python/paddle/distributed/cloud_utils.py): the
PaddleCloud environment (PADDLE_TRAINERS / POD_IP / PADDLE_TRAINER_ID ...)."""
import os

__all__ = ["use_paddlecloud", "get_trainers_num", "get_cluster_and_pod"]


def use_paddlecloud():
    return all(k in os.environ for k in ("PADDLE_TRAINERS", "POD_IP", "PADDLE_TRAINER_ID"))


def get_trainers_num():
    return int(os.environ.get("PADDLE_TRAINERS_NUM", "1"))


def get_cluster_and_pod(args=None):
    """(trainer endpoints, this trainer's index) from the environment"""
    eps = [e for e in os.environ.get("PADDLE_TRAINER_ENDPOINTS", "").split(",") if e]
    return eps, int(os.environ.get("PADDLE_TRAINER_ID", "0"))
