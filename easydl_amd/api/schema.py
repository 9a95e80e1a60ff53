"""Versioned wire schemas of the control plane.

The reference reserves a protobuf IDL (``easydl.proto`` -> ``easydl.pb.go``,
reference ``.pre-commit-config.yaml:31,63``) for the messages between the
trainer, the Brain and the operator.  No protoc exists in this environment and
every peer here is Python or C++ on one node, so the IDL is JSON Schema
(draft 2020-12 subset): one document per message kind, checked by the small
validator below at every process boundary that accepts JSON (CLI
``edl validate``, the operator's JobResource poll, the Brain service).

Kinds: ``ElasticJob``, ``JobResource`` (reference CRDs, Appendix A of SURVEY.md,
plus the MI355X resource fields), ``ResourcePlan`` (Brain output) and the Brain
RPC envelopes ``PlanRequest`` / ``PlanResponse``.
"""
from __future__ import annotations

SCHEMA_VERSION = "edl.mi355x/v1"
_API = {"enum": ["elastic.easydl.org/v1alpha1", "edl.mi355x/v1"]}
_NAME = {"type": "string", "minLength": 1}

RESOURCE = {
    "type": "object", "additionalProperties": False,
    "properties": {
        "cpu": {"type": "number", "minimum": 0}, "memory": {"type": "number", "minimum": 0},
        "disk": {"type": "number", "minimum": 0}, "gpu": {"type": "integer", "minimum": 0},
        "cu": {"type": "integer", "minimum": 0, "maximum": 256},
        "hbm_gb": {"type": "number", "minimum": 0, "maximum": 288},
    },
}
ROLE_RESOURCE = {"type": "object", "required": ["replicas"],
                 "properties": {"replicas": {"type": "integer", "minimum": 0}, "resource": RESOURCE}}
ROLE_SPEC = {"type": "object", "properties": {"image": {"type": ["string", "null"]},
                                              "command": {"type": ["string", "null"]}}}

SCHEMAS: dict[str, dict] = {
    "ElasticJob": {
        "type": "object", "required": ["kind", "metadata", "spec"],
        "properties": {
            "apiVersion": _API, "kind": {"const": "ElasticJob"},
            "metadata": {"type": "object", "required": ["name"], "properties": {"name": _NAME}},
            "spec": {"type": "object", "properties": {
                "command": {"type": "string"}, "image": {"type": ["string", "null"]},
                "parameter_server": ROLE_SPEC, "worker": ROLE_SPEC, "evaluator": ROLE_SPEC, "trainer": ROLE_SPEC,
                "mode": {"enum": ["allreduce", "ps"]}, "env": {"type": "object"},
                "min_workers": {"type": "integer", "minimum": 0}, "max_workers": {"type": "integer", "minimum": 1},
                "features": {"type": "object"}, "standby": {"type": "integer", "minimum": 0}}},
        },
    },
    "JobResource": {
        "type": "object", "required": ["kind", "spec"],
        "properties": {
            "apiVersion": _API, "kind": {"const": "JobResource"},
            "metadata": {"type": "object", "properties": {"name": _NAME}},
            "spec": {"type": "object", "required": ["selector"], "properties": {
                "selector": {"type": "object", "required": ["name"], "properties": {"name": _NAME}},
                "parameter_server": ROLE_RESOURCE, "worker": ROLE_RESOURCE, "evaluator": ROLE_RESOURCE,
                "resource_updation": {"type": "array", "items": {
                    "type": "object", "required": ["name", "resource"],
                    "properties": {"name": _NAME, "resource": RESOURCE}}},
                "bucket_mb": {"type": "number", "minimum": 0}, "ckpt_interval": {"type": "integer", "minimum": 0},
                "version": {"type": "integer", "minimum": 0}}},
        },
    },
    "ResourcePlan": {
        "type": "object", "required": ["roles"],
        "properties": {
            "roles": {"type": "object", "additionalProperties": ROLE_RESOURCE},
            "per_rank": {"type": "object"}, "bucket_mb": {"type": ["number", "null"], "minimum": 0},
            "ckpt_interval": {"type": ["integer", "null"], "minimum": 0}, "reason": {"type": "string"},
            "allreduce": {"type": ["object", "null"]},
        },
    },
    "PlanRequest": {
        "type": "object", "required": ["job", "kind"],
        "properties": {
            "schema": {"const": SCHEMA_VERSION}, "job": _NAME, "kind": {"enum": ["startup", "next"]},
            "features": {"type": "object"}, "current": {"type": ["object", "null"]},
            "metrics": {"type": "object"}, "comm": {"type": ["object", "null"]},
        },
    },
    "PlanResponse": {
        "type": "object", "required": ["plan"],
        "properties": {"schema": {"const": SCHEMA_VERSION}, "plan": {"type": ["object", "null"]},
                       "changed": {"type": "boolean"}},
    },
}

_TYPES = {"object": dict, "array": list, "string": str, "boolean": bool, "null": type(None)}


def _is(v, t: str) -> bool:
    if t == "integer":
        return isinstance(v, int) and not isinstance(v, bool)
    if t == "number":
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    return isinstance(v, _TYPES[t])


def errors(doc, schema: dict, path: str = "$") -> list[str]:
    """All violations of ``schema`` by ``doc`` (empty list = valid)."""
    out = []
    t = schema.get("type")
    if t is not None:
        types = t if isinstance(t, list) else [t]
        if not any(_is(doc, x) for x in types):
            return [f"{path}: expected {'/'.join(types)}, got {type(doc).__name__}"]
    if "const" in schema and doc != schema["const"]:
        out.append(f"{path}: must be {schema['const']!r}")
    if "enum" in schema and doc not in schema["enum"]:
        out.append(f"{path}: {doc!r} not in {schema['enum']}")
    if isinstance(doc, (int, float)) and not isinstance(doc, bool):
        if "minimum" in schema and doc < schema["minimum"]:
            out.append(f"{path}: {doc} < minimum {schema['minimum']}")
        if "maximum" in schema and doc > schema["maximum"]:
            out.append(f"{path}: {doc} > maximum {schema['maximum']}")
    if isinstance(doc, str) and len(doc) < schema.get("minLength", 0):
        out.append(f"{path}: shorter than {schema['minLength']}")
    if isinstance(doc, dict):
        props = schema.get("properties", {})
        for k in schema.get("required", []):
            if k not in doc:
                out.append(f"{path}: missing required '{k}'")
        extra = schema.get("additionalProperties", True)
        for k, v in doc.items():
            if k in props:
                out += errors(v, props[k], f"{path}.{k}")
            elif extra is False:
                out.append(f"{path}: unknown field '{k}'")
            elif isinstance(extra, dict):
                out += errors(v, extra, f"{path}.{k}")
    if isinstance(doc, list) and "items" in schema:
        for i, v in enumerate(doc):
            out += errors(v, schema["items"], f"{path}[{i}]")
    return out


def validate(doc: dict, kind: str | None = None) -> list[str]:
    """Validate a control-plane document; ``kind`` defaults to ``doc['kind']``."""
    kind = kind or (doc.get("kind") if isinstance(doc, dict) else None)
    if kind not in SCHEMAS:
        return [f"$: unknown message kind {kind!r}"]
    return errors(doc, SCHEMAS[kind])


def document(kind: str) -> dict:
    """The JSON Schema document of ``kind`` (what ``edl schema <kind>`` prints)."""
    return {"$schema": "https://json-schema.org/draft/2020-12/schema", "$id": f"{SCHEMA_VERSION}/{kind}",
            "title": kind, **SCHEMAS[kind]}
