"""Kubeflow PyTorchJob condition types and their mapping to DB states (C11;
``/root/reference/app/schemas/kubeflow_schemas.py:10-85``)."""
from __future__ import annotations

import logging
from enum import Enum

from .db import DatabaseStatusEnum

logger = logging.getLogger("ftc.schemas")


class KubeflowStatusEnum(str, Enum):
    created = "Created"        # accepted; pods not all started
    running = "Running"        # all replicas scheduled and running
    restarting = "Restarting"  # a replica failed and is being restarted (restartPolicy)
    succeeded = "Succeeded"
    suspended = "Suspended"    # Kueue holds the job (runPolicy.suspend)
    failed = "Failed"


_MAP = {
    KubeflowStatusEnum.suspended: DatabaseStatusEnum.queued,
    KubeflowStatusEnum.created: DatabaseStatusEnum.starting,
    KubeflowStatusEnum.running: DatabaseStatusEnum.running,
    KubeflowStatusEnum.restarting: DatabaseStatusEnum.restarting,
    KubeflowStatusEnum.succeeded: DatabaseStatusEnum.completed,
    KubeflowStatusEnum.failed: DatabaseStatusEnum.failed,
}


class TrainingJobStatus:
    running_states = [DatabaseStatusEnum.queued, DatabaseStatusEnum.starting, DatabaseStatusEnum.running,
                      DatabaseStatusEnum.restarting, KubeflowStatusEnum.created, KubeflowStatusEnum.running,
                      KubeflowStatusEnum.suspended, KubeflowStatusEnum.restarting]
    stopped_states = [DatabaseStatusEnum.completed, DatabaseStatusEnum.failed, DatabaseStatusEnum.canceled,
                      DatabaseStatusEnum.error, KubeflowStatusEnum.succeeded, KubeflowStatusEnum.failed]

    @classmethod
    def map_status(cls, kubeflow_status) -> DatabaseStatusEnum:
        try:
            return _MAP[KubeflowStatusEnum(kubeflow_status)]
        except (KeyError, ValueError):
            logger.error("job in unknown state: %s", kubeflow_status)
            return DatabaseStatusEnum.error

    @classmethod
    def is_running(cls, status) -> bool:
        return _status_value(status) in {_status_value(s) for s in cls.running_states}

    @classmethod
    def is_stopped(cls, status) -> bool:
        return _status_value(status) in {_status_value(s) for s in cls.stopped_states}


def _status_value(s) -> str:
    return s.value if isinstance(s, Enum) else str(s)
