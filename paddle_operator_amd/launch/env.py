"""The PaddleJob environment contract, read inside a rank's container.

Emitted by the controller (reference: controllers/paddlejob_helper.go:215-377,
SURVEY Appendix A) — POD_IP, PADDLE_TRAINER_ID, TRAINING_ROLE /
PADDLE_TRAINING_ROLE, the ConfigMap keys (PADDLE_TRAINER_ENDPOINTS,
PADDLE_TRAINERS_NUM, PADDLE_PSERVERS_IP_PORT_LIST, PADDLE_PORT, gloo keys) and
the elastic keys (PADDLE_ELASTIC_JOB_ID / _NP / _TIMEOUT / _SERVER) — plus
the pdo additions (PDO_JOB, PDO_ROLE, PDO_REPLICA_INDEX, PDO_REPLICAS,
HIP_VISIBLE_DEVICES from the agent/device plugin).

``JobEnv.torch_env()`` derives the torch.distributed contract (RANK,
WORLD_SIZE, MASTER_ADDR, MASTER_PORT, LOCAL_RANK) for the PyTorch-ROCm
launcher.  Port plan: each pod owns PADDLE_PORT … PADDLE_PORT+19; rank 0's
TCPStore (RCCL unique-id exchange) listens on PADDLE_PORT+1.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

STORE_PORT_OFFSET = 1


def _split(s: Optional[str]) -> List[str]:
    return [x for x in (s or "").split(",") if x]


@dataclass
class JobEnv:
    role: str = "TRAINER"
    trainer_id: int = 0
    pod_ip: str = "127.0.0.1"
    port: int = 2379
    trainer_endpoints: List[str] = field(default_factory=list)
    trainers_num: int = 1
    pserver_endpoints: List[str] = field(default_factory=list)
    heter_endpoints: List[str] = field(default_factory=list)
    with_gloo: int = 0
    gloo_endpoint: str = ""
    elastic_job_id: str = ""
    elastic_np: int = 0
    elastic_timeout: int = 60
    elastic_server: str = ""
    job: str = ""
    replica_index: int = 0
    replicas: int = 1
    pod_name: str = ""
    visible_devices: str = ""
    cp_size: int = 1

    @staticmethod
    def from_env(env: Optional[Dict[str, str]] = None) -> "JobEnv":
        e = env if env is not None else os.environ
        role = e.get("PADDLE_TRAINING_ROLE") or e.get("TRAINING_ROLE") or "TRAINER"
        tid = int(e.get("PADDLE_TRAINER_ID", e.get("RANK", "0")))
        eps = _split(e.get("PADDLE_TRAINER_ENDPOINTS"))
        num = int(e.get("PADDLE_TRAINERS_NUM", str(len(eps) or int(e.get("WORLD_SIZE", "1")))))
        return JobEnv(
            role=role,
            trainer_id=tid,
            pod_ip=e.get("POD_IP", e.get("PDO_POD_IP", "127.0.0.1")),
            port=int(e.get("PADDLE_PORT", "2379") or 2379),
            trainer_endpoints=eps,
            trainers_num=num,
            pserver_endpoints=_split(e.get("PADDLE_PSERVERS_IP_PORT_LIST")),
            heter_endpoints=_split(e.get("PADDLE_HETER_ENDPOINTS")),
            with_gloo=int(e.get("PADDLE_WITH_GLOO", "0") or 0),
            gloo_endpoint=e.get("PADDLE_GLOO_HTTP_ENDPOINT", ""),
            elastic_job_id=e.get("PADDLE_ELASTIC_JOB_ID", ""),
            elastic_np=int(e.get("PADDLE_ELASTIC_NP", "0") or 0),
            elastic_timeout=int(e.get("PADDLE_ELASTIC_TIMEOUT", "60") or 60),
            elastic_server=e.get("PADDLE_ELASTIC_SERVER", ""),
            job=e.get("PDO_JOB", ""),
            replica_index=int(e.get("PDO_REPLICA_INDEX", str(tid))),
            replicas=int(e.get("PDO_REPLICAS", str(num))),
            pod_name=e.get("HOSTNAME", ""),
            visible_devices=e.get("HIP_VISIBLE_DEVICES", ""),
            cp_size=int(e.get("PDO_CP_SIZE", "1") or 1),
        )

    # ------------------------------------------------------------------ modes
    @property
    def elastic(self) -> bool:
        return bool(self.elastic_job_id)

    @property
    def mode(self) -> str:
        if self.pserver_endpoints or self.role == "PSERVER":
            return "PS"
        if self.trainers_num > 1 or self.elastic:
            return "Collective"
        return "Single"

    def _host_port(self, ep: str):
        h, _, p = ep.rpartition(":")
        return h, int(p)

    def ps_world(self):
        """PS mode: ranks 0..P-1 are pservers, P..P+T-1 trainers, then heter workers."""
        P = len(self.pserver_endpoints)
        T = len(self.trainer_endpoints) or self.trainers_num
        H = len(self.heter_endpoints)
        if self.role == "PSERVER":
            rank = self.trainer_id
        elif self.role == "HETER":
            rank = P + T + self.trainer_id
        else:
            rank = P + self.trainer_id
        master = self.pserver_endpoints[0] if self.pserver_endpoints else f"{self.pod_ip}:{self.port}"
        return rank, P + T + H, master

    def torch_env(self, local_rank: int = 0, nproc_per_pod: int = 1) -> Dict[str, str]:
        if self.mode == "PS":
            rank, world, master = self.ps_world()
        else:
            rank = self.trainer_id * nproc_per_pod + local_rank
            world = self.trainers_num * nproc_per_pod
            master = self.trainer_endpoints[0] if self.trainer_endpoints else f"{self.pod_ip}:{self.port}"
        host, port = self._host_port(master)
        return {
            "RANK": str(rank),
            "WORLD_SIZE": str(world),
            "LOCAL_RANK": str(local_rank),
            "LOCAL_WORLD_SIZE": str(nproc_per_pod),
            "MASTER_ADDR": host,
            "MASTER_PORT": str(port + STORE_PORT_OFFSET),
        }

    def check_supported(self) -> None:
        """Context/sequence parallelism is an extension point only (SURVEY §5.7:
        the reference has none, no BASELINE config needs it — GPT-2-medium at
        ctx 1024 fits one MI355X).  ``PDO_CP_SIZE`` is read so a job that asks
        for it fails loudly instead of silently training data-parallel."""
        if self.cp_size != 1:
            raise NotImplementedError(f"PDO_CP_SIZE={self.cp_size}: context parallelism is not implemented "
                                      "(data parallel only; see SURVEY.md §5.7)")

    def kv_endpoints(self) -> str:
        return os.environ.get("PDO_KV", "") or self.elastic_server

    def job_key(self) -> str:
        if self.elastic_job_id:
            return self.elastic_job_id
        return (self.job or "default/job").replace("/", "-")
