"""Structural OpenAPI v3 schema of ``core/v1.PodTemplateSpec`` for the CRD,
plus the apiserver's structural pruning / validation over such a schema.

The reference's generated CRD embeds the full PodTemplateSpec schema for each
role (deploy/v1/crd.yaml:67-3146, :3156-6253, :6263-9340).  That gives two
behaviours a ``x-kubernetes-preserve-unknown-fields`` template lacks:

* **validation** — ``containers`` is required in a PodSpec and ``name`` in a
  Container, fields have types (a string ``replicas`` or a map ``command`` is
  rejected at admission, not when the pod is created);
* **structural pruning** — unknown fields are dropped on write, which is what
  silently removes the misspelled ``cleanPolicy`` of docs/user-guide.md:312
  (quirk D-9).

The schema is written from the core/v1 type table (field name → type), not
copied from generated YAML.  Deep, rarely templated leaves (projected /
downwardAPI / ephemeral volume sources, legacy in-tree volume plugins) are
``x-kubernetes-preserve-unknown-fields`` objects so nothing a user can write
today is lost.  ``prune`` / ``check`` implement the apiserver side; the
native local apiserver runs the same algorithm (csrc/core/schema.cpp) over the
same schema, compiled in from ``csrc/core/crd_schema.inc``.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

# ---------------------------------------------------------------- type helpers
S = {"type": "string"}
B = {"type": "boolean"}
I32 = {"type": "integer", "format": "int32"}
I64 = {"type": "integer", "format": "int64"}
QUANTITY = {"anyOf": [{"type": "integer"}, {"type": "string"}], "x-kubernetes-int-or-string": True,
            "pattern": r"^(\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))(([KMGTPE]i)|[numkMGTPE]|([eE](\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))))?$"}
INT_OR_STRING = {"anyOf": [{"type": "integer"}, {"type": "string"}], "x-kubernetes-int-or-string": True}
OPAQUE = {"type": "object", "x-kubernetes-preserve-unknown-fields": True}


def obj(props: Dict[str, Any], required: Optional[List[str]] = None, desc: str = "") -> dict:
    d: Dict[str, Any] = {"type": "object", "properties": props}
    if required:
        d["required"] = list(required)
    if desc:
        d["description"] = desc
    return d


def arr(items: dict) -> dict:
    return {"type": "array", "items": items}


def smap(v: dict = S) -> dict:
    return {"type": "object", "additionalProperties": v}


STRS = arr(S)
LOCAL_REF = obj({"name": S})
KEY_TO_PATH = obj({"key": S, "mode": I32, "path": S}, ["key", "path"])

# ---------------------------------------------------------------- selectors / affinity
REQUIREMENT = obj({"key": S, "operator": S, "values": STRS}, ["key", "operator"])
LABEL_SELECTOR = obj({"matchExpressions": arr(REQUIREMENT), "matchLabels": smap()})
NODE_SELECTOR_TERM = obj({"matchExpressions": arr(REQUIREMENT), "matchFields": arr(REQUIREMENT)})
POD_AFFINITY_TERM = obj({"labelSelector": LABEL_SELECTOR, "namespaceSelector": LABEL_SELECTOR,
                         "namespaces": STRS, "topologyKey": S}, ["topologyKey"])
WEIGHTED_POD_AFFINITY_TERM = obj({"podAffinityTerm": POD_AFFINITY_TERM, "weight": I32},
                                 ["podAffinityTerm", "weight"])
POD_AFFINITY = obj({"preferredDuringSchedulingIgnoredDuringExecution": arr(WEIGHTED_POD_AFFINITY_TERM),
                    "requiredDuringSchedulingIgnoredDuringExecution": arr(POD_AFFINITY_TERM)})
AFFINITY = obj({
    "nodeAffinity": obj({
        "preferredDuringSchedulingIgnoredDuringExecution": arr(
            obj({"preference": NODE_SELECTOR_TERM, "weight": I32}, ["preference", "weight"])),
        "requiredDuringSchedulingIgnoredDuringExecution": obj(
            {"nodeSelectorTerms": arr(NODE_SELECTOR_TERM)}, ["nodeSelectorTerms"]),
    }),
    "podAffinity": POD_AFFINITY,
    "podAntiAffinity": POD_AFFINITY,
})

# ---------------------------------------------------------------- security
SE_LINUX = obj({"level": S, "role": S, "type": S, "user": S})
SECCOMP = obj({"localhostProfile": S, "type": S}, ["type"])
WINDOWS = obj({"gmsaCredentialSpec": S, "gmsaCredentialSpecName": S, "hostProcess": B, "runAsUserName": S})
SECURITY_CONTEXT = obj({
    "allowPrivilegeEscalation": B, "capabilities": obj({"add": STRS, "drop": STRS}), "privileged": B,
    "procMount": S, "readOnlyRootFilesystem": B, "runAsGroup": I64, "runAsNonRoot": B, "runAsUser": I64,
    "seLinuxOptions": SE_LINUX, "seccompProfile": SECCOMP, "windowsOptions": WINDOWS})
POD_SECURITY_CONTEXT = obj({
    "fsGroup": I64, "fsGroupChangePolicy": S, "runAsGroup": I64, "runAsNonRoot": B, "runAsUser": I64,
    "seLinuxOptions": SE_LINUX, "seccompProfile": SECCOMP, "supplementalGroups": arr(I64),
    "sysctls": arr(obj({"name": S, "value": S}, ["name", "value"])), "windowsOptions": WINDOWS})

# ---------------------------------------------------------------- container
EXEC_ACTION = obj({"command": STRS})
HTTP_GET = obj({"host": S, "httpHeaders": arr(obj({"name": S, "value": S}, ["name", "value"])), "path": S,
                "port": INT_OR_STRING, "scheme": S}, ["port"])
TCP_SOCKET = obj({"host": S, "port": INT_OR_STRING}, ["port"])
PROBE = obj({"exec": EXEC_ACTION, "failureThreshold": I32, "grpc": obj({"port": I32, "service": S}, ["port"]),
             "httpGet": HTTP_GET, "initialDelaySeconds": I32, "periodSeconds": I32, "successThreshold": I32,
             "tcpSocket": TCP_SOCKET, "terminationGracePeriodSeconds": I64, "timeoutSeconds": I32})
HANDLER = obj({"exec": EXEC_ACTION, "httpGet": HTTP_GET, "tcpSocket": TCP_SOCKET})
ENV_VAR = obj({"name": S, "value": S, "valueFrom": obj({
    "configMapKeyRef": obj({"key": S, "name": S, "optional": B}, ["key"]),
    "fieldRef": obj({"apiVersion": S, "fieldPath": S}, ["fieldPath"]),
    "resourceFieldRef": obj({"containerName": S, "divisor": QUANTITY, "resource": S}, ["resource"]),
    "secretKeyRef": obj({"key": S, "name": S, "optional": B}, ["key"]),
})}, ["name"])
ENV_FROM = obj({"configMapRef": obj({"name": S, "optional": B}), "prefix": S,
                "secretRef": obj({"name": S, "optional": B})})
RESOURCES = obj({"limits": smap(QUANTITY), "requests": smap(QUANTITY)})
CONTAINER_PROPS = {
    "args": STRS, "command": STRS, "env": arr(ENV_VAR), "envFrom": arr(ENV_FROM), "image": S,
    "imagePullPolicy": S, "lifecycle": obj({"postStart": HANDLER, "preStop": HANDLER}),
    "livenessProbe": PROBE, "name": S,
    "ports": arr(obj({"containerPort": I32, "hostIP": S, "hostPort": I32, "name": S, "protocol": S},
                     ["containerPort"])),
    "readinessProbe": PROBE, "resources": RESOURCES, "securityContext": SECURITY_CONTEXT, "startupProbe": PROBE,
    "stdin": B, "stdinOnce": B, "terminationMessagePath": S, "terminationMessagePolicy": S, "tty": B,
    "volumeDevices": arr(obj({"devicePath": S, "name": S}, ["devicePath", "name"])),
    "volumeMounts": arr(obj({"mountPath": S, "mountPropagation": S, "name": S, "readOnly": B, "subPath": S,
                             "subPathExpr": S}, ["mountPath", "name"])),
    "workingDir": S,
}
CONTAINER = obj(CONTAINER_PROPS, ["name"])
EPHEMERAL_CONTAINER = obj(dict(CONTAINER_PROPS, targetContainerName=S), ["name"])

# ---------------------------------------------------------------- volumes
LEGACY_SOURCES = ("awsElasticBlockStore", "azureDisk", "azureFile", "cephfs", "cinder", "downwardAPI", "ephemeral",
                  "fc", "flexVolume", "flocker", "gcePersistentDisk", "gitRepo", "glusterfs", "iscsi",
                  "photonPersistentDisk", "portworxVolume", "projected", "quobyte", "rbd", "scaleIO", "storageos",
                  "vsphereVolume")
VOLUME_PROPS = {
    "name": S,
    "configMap": obj({"defaultMode": I32, "items": arr(KEY_TO_PATH), "name": S, "optional": B}),
    "secret": obj({"defaultMode": I32, "items": arr(KEY_TO_PATH), "optional": B, "secretName": S}),
    "emptyDir": obj({"medium": S, "sizeLimit": QUANTITY}),
    "hostPath": obj({"path": S, "type": S}, ["path"]),
    "persistentVolumeClaim": obj({"claimName": S, "readOnly": B}, ["claimName"]),
    "nfs": obj({"path": S, "readOnly": B, "server": S}, ["path", "server"]),
    "csi": obj({"driver": S, "fsType": S, "nodePublishSecretRef": LOCAL_REF, "readOnly": B,
                "volumeAttributes": smap()}, ["driver"]),
}
VOLUME_PROPS.update({k: OPAQUE for k in LEGACY_SOURCES})
VOLUME = obj(VOLUME_PROPS, ["name"])

# ---------------------------------------------------------------- pod
POD_SPEC = obj({
    "activeDeadlineSeconds": I64, "affinity": AFFINITY, "automountServiceAccountToken": B,
    "containers": arr(CONTAINER),
    "dnsConfig": obj({"nameservers": STRS, "options": arr(obj({"name": S, "value": S})), "searches": STRS}),
    "dnsPolicy": S, "enableServiceLinks": B, "ephemeralContainers": arr(EPHEMERAL_CONTAINER),
    "hostAliases": arr(obj({"hostnames": STRS, "ip": S})), "hostIPC": B, "hostNetwork": B, "hostPID": B,
    "hostname": S, "imagePullSecrets": arr(LOCAL_REF), "initContainers": arr(CONTAINER), "nodeName": S,
    "nodeSelector": smap(), "os": obj({"name": S}, ["name"]), "overhead": smap(QUANTITY),
    "preemptionPolicy": S, "priority": I32, "priorityClassName": S,
    "readinessGates": arr(obj({"conditionType": S}, ["conditionType"])), "restartPolicy": S,
    "runtimeClassName": S, "schedulerName": S, "securityContext": POD_SECURITY_CONTEXT, "serviceAccount": S,
    "serviceAccountName": S, "setHostnameAsFQDN": B, "shareProcessNamespace": B, "subdomain": S,
    "terminationGracePeriodSeconds": I64,
    "tolerations": arr(obj({"effect": S, "key": S, "operator": S, "tolerationSeconds": I64, "value": S})),
    "topologySpreadConstraints": arr(obj({"labelSelector": LABEL_SELECTOR, "maxSkew": I32, "minDomains": I32,
                                          "topologyKey": S, "whenUnsatisfiable": S},
                                         ["maxSkew", "topologyKey", "whenUnsatisfiable"])),
    "volumes": arr(VOLUME),
}, ["containers"])
EMBEDDED_META = obj({"annotations": smap(), "finalizers": STRS, "labels": smap(), "name": S, "namespace": S})


def pod_template_schema() -> dict:
    return obj({"metadata": EMBEDDED_META, "spec": POD_SPEC}, desc="Template specifies the podspec of a server")


# ---------------------------------------------------------------- apiserver side
def _preserve(schema: dict) -> bool:
    return bool(schema.get("x-kubernetes-preserve-unknown-fields"))


def prune(value: Any, schema: dict, root: bool = True) -> Any:
    """Structural pruning (k8s apiextensions): drop object fields the schema
    does not declare, unless the node preserves unknown fields.  ``metadata``
    of the root object is the apiserver's and never pruned here."""
    if isinstance(value, dict) and (schema.get("type") == "object" or "properties" in schema):
        props = schema.get("properties")
        addl = schema.get("additionalProperties")
        out = {}
        for k, v in value.items():
            if root and k == "metadata":
                out[k] = v
            elif props is not None and k in props:
                out[k] = prune(v, props[k], False)
            elif isinstance(addl, dict):
                out[k] = prune(v, addl, False)
            elif _preserve(schema):
                out[k] = v
        return out
    if isinstance(value, list) and isinstance(schema.get("items"), dict):
        return [prune(v, schema["items"], False) for v in value]
    return value


def _type_ok(value: Any, schema: dict) -> bool:
    if "anyOf" in schema:
        return any(_type_ok(value, s) for s in schema["anyOf"])
    t = schema.get("type")
    if t is None:
        return True
    if t == "object":
        return isinstance(value, dict)
    if t == "array":
        return isinstance(value, list)
    if t == "string":
        return isinstance(value, str)
    if t == "integer":
        return isinstance(value, int) and not isinstance(value, bool)
    if t == "number":
        return isinstance(value, (int, float)) and not isinstance(value, bool)
    if t == "boolean":
        return isinstance(value, bool)
    return True


def check(value: Any, schema: dict, path: str = "") -> List[str]:
    """Type + required-field errors (``path: message``), as the apiserver's
    422 Invalid details.  ``null`` is accepted for optional fields (omitempty)."""
    errs: List[str] = []
    if value is None:
        return errs
    if not _type_ok(value, schema):
        want = schema.get("type") or "int-or-string"
        return [f"{path or '<root>'}: Invalid value: must be of type {want}"]
    if isinstance(value, dict):
        for r in schema.get("required") or []:
            if r not in value or value[r] is None:
                errs.append(f"{path + '.' if path else ''}{r}: Required value")
        props = schema.get("properties") or {}
        addl = schema.get("additionalProperties")
        for k, v in value.items():
            sub = f"{path}.{k}" if path else k
            if k in props:
                errs += check(v, props[k], sub)
            elif isinstance(addl, dict):
                errs += check(v, addl, sub)
    elif isinstance(value, list) and isinstance(schema.get("items"), dict):
        for i, v in enumerate(value):
            errs += check(v, schema["items"], f"{path}[{i}]")
    return errs
