"""PaddleJob API (``batch.paddlepaddle.org/v1``) — Python mirror of the schema.

Field names, enum strings and omitempty behaviour are those of the reference
CRD (``/root/reference/api/v1/paddlejob_types.go:25-281``); the native
control plane (``csrc/core/api.h``) is the source of truth at run time, this
module gives Python users typed builders and pydantic validation.
"""
from __future__ import annotations

import copy
from typing import Any, Dict, List, Optional

from pydantic import BaseModel, ConfigDict, Field

GROUP = "batch.paddlepaddle.org"
VERSION = "v1"
API_VERSION = f"{GROUP}/{VERSION}"
KIND = "PaddleJob"
PLURAL = "paddlejobs"
SHORT_NAME = "pdj"

# labels / annotations (paddlejob_types.go:29-35)
LABEL_RESOURCE_NAME = "paddle-res-name"
LABEL_RESOURCE_TYPE = "paddle-res-type"
ANNOTATION_RESOURCE = "paddle-resource"
ANNOTATION_HOST_PORT = "host-port"
FINALIZER = "finalizers.paddlepaddle.org"

ROLE_PS, ROLE_WORKER, ROLE_HETER = "ps", "worker", "heter"
ROLE_ORDER = (ROLE_PS, ROLE_WORKER, ROLE_HETER)
TRAINING_ROLE = {ROLE_PS: "PSERVER", ROLE_WORKER: "TRAINER", ROLE_HETER: "HETER"}

PADDLE_PORT = 2379
PORTS_PER_POD = 20


class Phase:
    Starting = "Starting"
    Pending = "Pending"
    Scaling = "Scaling"
    Aborting = "Aborting"
    Aborted = "Aborted"
    Running = "Running"
    Restarting = "Restarting"
    Completing = "Completing"
    Completed = "Completed"
    Terminating = "Terminating"
    Terminated = "Terminated"
    Failed = "Failed"
    Succeed = "Succeed"
    Unknown = "Unknown"


class Mode:
    PS = "PS"
    Collective = "Collective"
    Single = "Single"


class CleanPodPolicy:
    Always = "Always"
    Never = "Never"
    OnFailure = "OnFailure"
    OnCompletion = "OnCompletion"


class Intranet:
    PodIP = "PodIP"
    Service = "Service"
    Host = "Host"


class ElasticStatus:
    NONE = "NONE"
    DOING = "DOING"
    DONE = "DONE"
    ERROR = "ERROR"


AMD_GPU = "amd.com/gpu"


class _Model(BaseModel):
    model_config = ConfigDict(populate_by_name=True, extra="allow")


class ResourceSpec(_Model):
    replicas: int
    requests: Optional[int] = None
    limits: Optional[int] = None
    template: Dict[str, Any] = Field(default_factory=dict)


class SchedulingPolicy(_Model):
    minAvailable: Optional[int] = None
    queue: Optional[str] = None
    priorityClass: Optional[str] = None
    minResources: Optional[Dict[str, Any]] = None


class PaddleJobSpec(_Model):
    cleanPodPolicy: Optional[str] = None
    schedulingPolicy: Optional[SchedulingPolicy] = None
    intranet: Optional[str] = None
    withGloo: Optional[int] = None
    ps: Optional[ResourceSpec] = None
    worker: Optional[ResourceSpec] = None
    heter: Optional[ResourceSpec] = None
    elastic: Optional[int] = None


class ResourceStatus(_Model):
    pending: int = 0
    starting: int = 0
    running: int = 0
    failed: int = 0
    succeeded: int = 0
    unknown: int = 0
    refs: List[Dict[str, Any]] = Field(default_factory=list)


class PaddleJobStatus(_Model):
    phase: Optional[str] = None
    mode: Optional[str] = None
    ps: Optional[ResourceStatus] = None
    worker: Optional[ResourceStatus] = None
    heter: Optional[ResourceStatus] = None
    elastic: Optional[str] = None
    startTime: Optional[str] = None
    completionTime: Optional[str] = None
    observedGeneration: Optional[int] = None


class PaddleJob(_Model):
    apiVersion: str = API_VERSION
    kind: str = KIND
    metadata: Dict[str, Any] = Field(default_factory=dict)
    spec: PaddleJobSpec = Field(default_factory=PaddleJobSpec)
    status: Optional[PaddleJobStatus] = None

    def to_dict(self) -> dict:
        return self.model_dump(exclude_none=True)


def validate(obj: dict) -> PaddleJob:
    """Parse + schema-validate a PaddleJob dict: the typed model (raises
    pydantic.ValidationError) and then the CRD's structural schema, role
    templates included, as the apiserver would at admission (ValueError)."""
    job = PaddleJob.model_validate(obj)
    from .crd import openapi_schema
    from .podschema import check
    errs = check(obj, openapi_schema())
    if errs:
        raise ValueError(f"{len(errs)} structural validation error(s): " + "; ".join(errs))
    return job


def container(name: str, command: List[str], image: str = "pdo/launcher:rocm", gpus: int = 0,
              env: Optional[Dict[str, str]] = None, args: Optional[List[str]] = None,
              cpu: Optional[str] = None, memory: Optional[str] = None) -> dict:
    c: Dict[str, Any] = {"name": name, "image": image, "command": list(command)}
    if args:
        c["args"] = list(args)
    if env:
        c["env"] = [{"name": k, "value": str(v)} for k, v in env.items()]
    res: Dict[str, Any] = {}
    if gpus:
        res.setdefault("limits", {})[AMD_GPU] = gpus
    if cpu:
        res.setdefault("requests", {})["cpu"] = cpu
    if memory:
        res.setdefault("requests", {})["memory"] = memory
    if res:
        c["resources"] = res
    return c


def role(replicas: int, containers: List[dict], **pod_spec) -> dict:
    spec = {"containers": containers}
    spec.update(pod_spec)
    return {"replicas": replicas, "template": {"spec": spec}}


def paddlejob(name: str, namespace: str = "default", *, ps: Optional[dict] = None,
              worker: Optional[dict] = None, heter: Optional[dict] = None,
              clean_pod_policy: Optional[str] = None, intranet: Optional[str] = None,
              with_gloo: Optional[int] = None, elastic: Optional[int] = None,
              scheduling_policy: Optional[dict] = None, labels: Optional[dict] = None) -> dict:
    spec: Dict[str, Any] = {}
    if clean_pod_policy is not None:
        spec["cleanPodPolicy"] = clean_pod_policy
    if scheduling_policy is not None:
        spec["schedulingPolicy"] = scheduling_policy
    if intranet is not None:
        spec["intranet"] = intranet
    if with_gloo is not None:
        spec["withGloo"] = with_gloo
    for k, v in (("ps", ps), ("worker", worker), ("heter", heter)):
        if v is not None:
            spec[k] = copy.deepcopy(v)
    if elastic is not None:
        spec["elastic"] = elastic
    md: Dict[str, Any] = {"name": name, "namespace": namespace}
    if labels:
        md["labels"] = dict(labels)
    return {"apiVersion": API_VERSION, "kind": KIND, "metadata": md, "spec": spec}
