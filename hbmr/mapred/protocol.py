"""Wire objects of the JobTracker <-> TaskTracker protocol.

Plain dataclasses that serialise to msgpack-able dicts, so the same objects go
through an in-process call or the TCP RPC (:mod:`hbmr.mapred.rpc`).

Mirrors InterTrackerProtocol.heartbeat (hadoop-1.0.3/src/mapred/org/apache/hadoop/
mapred/InterTrackerProtocol.java:103) with the GPU fork's additions made
first-class: a tracker reports CPU map slots and, per GPU device, its GPU map
slots (TaskTrackerStatus.java:63-65, 394-404 kept only two ints; here every
device is explicit, which is what availableGPUDevices() reconstructed at
TaskTrackerStatus.java:536-551), every task carries ``run_on_gpu`` and
``gpu_device_id`` (Task.java:169-207, TaskStatus.java:66-67) and the device id
really reaches the task (fixes SURVEY.md B1).  The protocol version is bumped
whenever the wire format changes (the fork did not: B9).
"""
from __future__ import annotations

from dataclasses import dataclass, field

PROTOCOL_VERSION = 5

# task states (TaskStatus.State)
UNASSIGNED = "UNASSIGNED"
RUNNING = "RUNNING"
COMMIT_PENDING = "COMMIT_PENDING"
SUCCEEDED = "SUCCEEDED"
FAILED = "FAILED"
KILLED = "KILLED"
FAILED_UNCLEAN = "FAILED_UNCLEAN"

TERMINAL = (SUCCEEDED, FAILED, KILLED)


@dataclass
class TaskStatus:
    attempt_id: str
    is_map: bool
    state: str = UNASSIGNED
    progress: float = 0.0
    run_on_gpu: bool = False
    gpu_device_id: int = -1
    start_time: float = 0.0
    finish_time: float = 0.0
    diagnostic: str = ""
    counters: dict = field(default_factory=dict)
    output: dict = field(default_factory=dict)   # where the map output lives
    status: str = ""
    # time spent on the device (HIP events) for GPU tasks, seconds
    device_time: float = 0.0

    def runOnCPU(self):  # noqa: N802
        return not self.run_on_gpu

    def to_dict(self):
        return dict(self.__dict__)   # shallow: fields are plain values / dicts

    @classmethod
    def from_dict(cls, d):
        return cls(**d)


@dataclass
class GpuDeviceStatus:
    device: int
    max_slots: int
    running: int = 0
    queued: int = 0
    hbm_total: int = 0
    hbm_free: int = 0
    name: str = ""


@dataclass
class TaskTrackerStatus:
    tracker_name: str
    host: str
    http_port: int = 0
    max_cpu_map_slots: int = 2
    max_reduce_slots: int = 1
    gpus: list = field(default_factory=list)        # [GpuDeviceStatus as dict]
    task_reports: list = field(default_factory=list)  # [TaskStatus as dict]
    cached_splits_added: list = field(default_factory=list)    # [(split_key, device)]
    cached_splits_removed: list = field(default_factory=list)
    healthy: bool = True
    health_report: str = ""
    rank: int = 0
    world_size: int = 1
    cpu_threads: int = 1
    # GPU map attempts that completed as one batch (one HIP event pair):
    # [{"attempts": [...], "device_time": s, "finish_time": t, "counters": {...},
    #   "output": {...}}] — the compact form of len(attempts) SUCCEEDED reports
    bulk_reports: list = field(default_factory=list)
    # succeeded map attempts whose output was lost (their GPU worker died)
    lost_outputs: list = field(default_factory=list)
    # the tracker's GPU worker process died and its collective peers must be
    # restarted with it (world > 1): the JobTracker answers restart_gpu_worker
    gpu_worker_lost: bool = False
    # the tracker's count of wakeup() notifications when this status was built:
    # a wakeup with a higher count carries news this heartbeat does not have,
    # so the JobTracker must not swallow it in the long-poll
    notify_seq: int = 0

    @property
    def max_gpu_map_slots(self):
        return sum(g["max_slots"] for g in self.gpus)

    def to_dict(self):
        return dict(self.__dict__)   # shallow: fields are plain values / dicts

    @classmethod
    def from_dict(cls, d):
        return cls(**d)


@dataclass
class TaskSpec:
    """Everything a tracker needs to run one attempt (LaunchTaskAction payload)."""
    attempt_id: str
    job_id: str
    is_map: bool
    partition: int
    run_on_gpu: bool = False
    gpu_device_id: int = -1
    split: dict = field(default_factory=dict)     # serialised split (kind + fields)
    num_maps: int = 0
    num_reduces: int = 0
    # classic reduce: [(map_attempt_id, output dict)] ; collective reduce: committed map attempts
    map_outputs: list = field(default_factory=list)
    collective: bool = False
    conf: dict | None = None                      # job conf (sent once per tracker per job)
    profile_fraction: float = 0.0                 # >0: sampled CPU profiling probe
    # map attempt of a staged job: held on the tracker until job ``gate``'s
    # collective reduce there has enqueued its result (JobTracker pre-staging)
    gate: str | None = None
    # collective reduce launched before its maps finished: ``map_outputs`` lists
    # the expected attempts, some still running; it waits for them to launch
    expect: bool = False

    def to_dict(self):
        return dict(self.__dict__)   # shallow: fields are plain values / dicts

    @classmethod
    def from_dict(cls, d):
        return cls(**d)


# heartbeat response actions ---------------------------------------------------
def launch_action(spec: TaskSpec):
    return {"type": "launch", "task": spec.to_dict()}


# {"type": "launch_batch", "job_id", "run_on_gpu", "device", "num_maps",
#  "num_reduces", "collective", "tasks": [[attempt_id, partition, split], ...],
#  "conf"?, "gate"?} — built by JobTracker.launch_gpu_batch


def kill_task_action(attempt_id: str):
    return {"type": "kill_task", "attempt_id": attempt_id}


def kill_job_action(job_id: str):
    return {"type": "kill_job", "job_id": job_id}


def commit_action(attempt_id: str):
    return {"type": "commit", "attempt_id": attempt_id}


def restart_gpu_worker_action(generation: int):
    return {"type": "restart_gpu_worker", "generation": generation}


def close_gate_action(job_id: str):
    """Job ``job_id``'s collective reduce restarts: forget its opened gate, so
    re-launched staged maps wait for the new reduce (hbmr/gpu/gates.py)."""
    return {"type": "close_gate", "job_id": job_id}


def reinit_action():
    return {"type": "reinit"}


def shutdown_action():
    return {"type": "shutdown"}
