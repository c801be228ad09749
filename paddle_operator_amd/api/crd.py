"""CustomResourceDefinition generator for PaddleJob.

Produces the apiextensions.k8s.io/v1 CRD (k8s ≥ 1.16) and the v1beta1 CRD
(k8s ≤ 1.15) with the identity of the reference's generated manifests
(``deploy/v1/crd.yaml:1-43,9465-9466``): group batch.paddlepaddle.org,
version v1, kind PaddleJob, plural paddlejobs, short name pdj, printer
columns Status/Mode/Age and the status subresource.

Role templates carry a structural corev1.PodTemplateSpec schema
(api/podschema.py) like the reference's embedded one, so the apiserver
validates them (containers required, container name required, field types)
and prunes unknown fields at admission.  Enum fields stay plain strings like
the reference (Appendix D-9).

usage: python -m paddle_operator_amd.api.crd [--v1beta1] > crd.yaml
"""
from __future__ import annotations

import argparse
import sys

import yaml

from . import types as T
from .podschema import pod_template_schema


def _int(desc, **kw):
    d = {"type": "integer", "description": desc}
    d.update(kw)
    return d


def _str(desc, **kw):
    d = {"type": "string", "description": desc}
    d.update(kw)
    return d


def resource_spec_schema(role: str) -> dict:
    return {
        "type": "object",
        "description": f"{role} describes the spec of {role} base on pod template",
        "required": ["replicas"],
        "properties": {
            "replicas": _int("Replicas replica"),
            "requests": _int("Requests set the minimal replicas of server to be run"),
            "limits": _int("Limits set the maximal replicas of server to be run, elastic is auto enabled "
                           "if limits is set larger than 0"),
            "template": pod_template_schema(),
        },
    }


def resource_status_schema(role: str) -> dict:
    props = {k: _int(k.capitalize()) for k in ("pending", "starting", "running", "failed",
                                                "succeeded", "unknown")}
    props["refs"] = {
        "type": "array",
        "description": "A list of pointer to pods",
        "items": {
            "type": "object",
            "properties": {k: _str(k) for k in ("apiVersion", "fieldPath", "kind", "name", "namespace",
                                                  "resourceVersion", "uid")},
        },
    }
    return {"type": "object", "description": f"ResourceStatues of {role}", "properties": props}


def openapi_schema() -> dict:
    spec = {
        "type": "object",
        "description": "PaddleJobSpec defines the desired state of PaddleJob",
        "properties": {
            "cleanPodPolicy": _str("CleanPodPolicy defines whether to clean pod after job finished"),
            "schedulingPolicy": {
                "type": "object",
                "description": "SchedulingPolicy defines the policy related to scheduling, for volcano",
                "properties": {
                    "minAvailable": _int("", format="int32"),
                    "queue": _str(""),
                    "priorityClass": _str(""),
                    "minResources": {
                        "type": "object",
                        "additionalProperties": {
                            "anyOf": [{"type": "integer"}, {"type": "string"}],
                            "x-kubernetes-int-or-string": True,
                        },
                    },
                },
            },
            "intranet": _str("Intranet defines the communication mode inter pods : PodIP, Service or Host"),
            "withGloo": _int("WithGloo indicate whether enable gloo, 0/1/2 for disable/enable for "
                             "worker/enable for server"),
            "ps": resource_spec_schema("ps"),
            "worker": resource_spec_schema("worker"),
            "heter": resource_spec_schema("heter"),
            "elastic": _int("Elastic indicate the elastic level"),
        },
    }
    status = {
        "type": "object",
        "description": "PaddleJobStatus defines the observed state of PaddleJob",
        "properties": {
            "phase": _str("The phase of PaddleJob."),
            "mode": _str("Mode indicates in which the PaddleJob run with : PS/Collective/Single"),
            "ps": resource_status_schema("ps"),
            "worker": resource_status_schema("worker"),
            "heter": resource_status_schema("heter"),
            "elastic": _str("Elastic"),
            "startTime": _str("StartTime indicate when the job started", format="date-time"),
            "completionTime": _str("CompletionTime indicate when the job completed/failed", format="date-time"),
            "observedGeneration": _int(""),
        },
    }
    return {
        "type": "object",
        "description": "PaddleJob is the Schema for the paddlejobs API",
        "properties": {
            "apiVersion": _str("APIVersion defines the versioned schema of this representation of an object."),
            "kind": _str("Kind is a string value representing the REST resource this object represents."),
            "metadata": {"type": "object"},
            "spec": spec,
            "status": status,
        },
    }


PRINTER_COLUMNS = [
    ("Status", "string", ".status.phase"),
    ("Mode", "string", ".status.mode"),
    ("Age", "date", ".metadata.creationTimestamp"),
]


def crd_v1() -> dict:
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{T.PLURAL}.{T.GROUP}",
                     "annotations": {"controller-gen.kubebuilder.io/version": "pdo-crdgen"}},
        "spec": {
            "group": T.GROUP,
            "names": {"kind": T.KIND, "listKind": T.KIND + "List", "plural": T.PLURAL,
                      "shortNames": [T.SHORT_NAME], "singular": T.KIND.lower()},
            "scope": "Namespaced",
            "versions": [{
                "name": T.VERSION,
                "served": True,
                "storage": True,
                "additionalPrinterColumns": [{"name": n, "type": t, "jsonPath": p}
                                             for n, t, p in PRINTER_COLUMNS],
                "schema": {"openAPIV3Schema": openapi_schema()},
                "subresources": {"status": {}},
            }],
        },
    }


def crd_v1beta1() -> dict:
    return {
        "apiVersion": "apiextensions.k8s.io/v1beta1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{T.PLURAL}.{T.GROUP}"},
        "spec": {
            "group": T.GROUP,
            "names": {"kind": T.KIND, "listKind": T.KIND + "List", "plural": T.PLURAL,
                      "shortNames": [T.SHORT_NAME], "singular": T.KIND.lower()},
            "scope": "Namespaced",
            "additionalPrinterColumns": [{"name": n, "type": t, "JSONPath": p} for n, t, p in PRINTER_COLUMNS],
            "subresources": {"status": {}},
            "validation": {"openAPIV3Schema": openapi_schema()},
            "version": T.VERSION,
            "versions": [{"name": T.VERSION, "served": True, "storage": True}],
        },
    }


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--v1beta1", action="store_true")
    a = ap.parse_args(argv)
    doc = crd_v1beta1() if a.v1beta1 else crd_v1()
    sys.stdout.write("---\n" + yaml.safe_dump(doc, sort_keys=False))


if __name__ == "__main__":
    main()
