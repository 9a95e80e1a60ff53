"""Brain as a service: HTTP/JSON endpoints (no protoc/gRPC codegen exists in this
environment — SURVEY.md §2.3 I2) plus an in-process client.

Endpoints (POST, JSON in/out):
    /startup_plan   {features}                      -> ResourcePlan
    /next_plan      {features, plan, metrics, comm} -> ResourcePlan | null
    /inventory      {}                              -> NodeInventory
Run: ``python -m easydl_amd.brain.service --port 8808``.
"""
from __future__ import annotations

import argparse
import json
import threading
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from easydl_amd.api.spec import ResourcePlan
from easydl_amd.brain.collectors import NodeInventory, host_inventory
from easydl_amd.brain.planner import JobFeatures, Planner


class BrainClient:
    """Talks to a Brain service at ``url``, or runs the planner in-process when url is None."""

    def __init__(self, url: str | None = None, planner: Planner | None = None, inventory=None):
        self.url = url
        self.planner = planner or Planner()
        self._inventory = inventory

    def inventory(self, telemetry: bool = False) -> NodeInventory:
        if self._inventory is not None:
            return self._inventory() if callable(self._inventory) else self._inventory
        return host_inventory(telemetry)

    def _post(self, path: str, body: dict):
        req = urllib.request.Request(self.url.rstrip("/") + path, data=json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=30) as r:
            return json.loads(r.read().decode() or "null")

    def startup_plan(self, features: dict) -> ResourcePlan:
        if self.url:
            return ResourcePlan.from_dict(self._post("/startup_plan", {"features": features}))
        return self.planner.startup_plan(JobFeatures.from_dict(features), self.inventory())

    def next_plan(self, features: dict, plan: ResourcePlan, metrics: dict,
                  comm: dict | None = None) -> ResourcePlan | None:
        if self.url:
            r = self._post("/next_plan", {"features": features, "plan": plan.to_dict(), "metrics": metrics,
                                          "comm": comm})
            return None if r is None else ResourcePlan.from_dict(r)
        return self.planner.next_plan(JobFeatures.from_dict(features), self.inventory(True), plan, metrics, comm)


class _Handler(BaseHTTPRequestHandler):
    planner: Planner = None

    def log_message(self, *a):
        pass

    def do_POST(self):
        n = int(self.headers.get("Content-Length", 0))
        body = json.loads(self.rfile.read(n).decode() or "{}")
        try:
            from easydl_amd.api.schema import errors, SCHEMAS
            if self.path in ("/startup_plan", "/next_plan"):
                bad = errors(body.get("features", {}), {"type": "object"})
                if self.path == "/next_plan":
                    bad += errors(body.get("plan"), SCHEMAS["ResourcePlan"], "$.plan")
                if bad:
                    data = json.dumps({"error": "schema", "details": bad}).encode()
                    self.send_response(400)
                    self.send_header("Content-Type", "application/json")
                    self.send_header("Content-Length", str(len(data)))
                    self.end_headers()
                    self.wfile.write(data)
                    return
            if self.path == "/startup_plan":
                out = self.planner.startup_plan(JobFeatures.from_dict(body.get("features")), host_inventory()).to_dict()
            elif self.path == "/next_plan":
                p = self.planner.next_plan(JobFeatures.from_dict(body.get("features")), host_inventory(True),
                                           ResourcePlan.from_dict(body["plan"]), body.get("metrics") or {},
                                           body.get("comm"))
                out = None if p is None else p.to_dict()
            elif self.path == "/inventory":
                out = host_inventory(True).to_dict()
            else:
                self.send_error(404)
                return
            data = json.dumps(out).encode()
            self.send_response(200)
        except Exception as e:  # pragma: no cover
            data = json.dumps({"error": str(e)}).encode()
            self.send_response(500)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)


def serve(port: int = 0, host: str = "127.0.0.1", planner: Planner | None = None):
    handler = type("H", (_Handler,), {"planner": planner or Planner()})
    srv = ThreadingHTTPServer((host, port), handler)
    t = threading.Thread(target=srv.serve_forever, daemon=True, name="edl-brain")
    t.start()
    return srv


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=8808)
    ap.add_argument("--host", default="127.0.0.1")
    a = ap.parse_args(argv)
    srv = serve(a.port, a.host)
    print(json.dumps({"brain_port": srv.server_address[1]}), flush=True)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        pass


if __name__ == "__main__":
    main()
