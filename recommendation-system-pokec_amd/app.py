"""app.py — HTTP front end over the engine's api_cli (the serving half).

The reference's wrapper is python/app.py:1-162: a FastAPI app that starts the C++ api_cli as
a child process, waits for its READY line, and forwards one "USER <uid>" line per request
under a lock (the CLI is single-threaded; the caller serialises).  Its
routes are kept, with the same paths, parameters and JSON:

    GET /                               a small HTML page (the reference renders templates/index.html)
    GET /health                         {"status": "ok", "load_users": N}            (app.py:104-106)
    GET /api/user/{uid}                 the api_cli JSON line for "USER uid"         (app.py:108-120)
    GET /api/recommend/{kind}/{uid}?topk=20, kind in graph|collab|interest|clubs:
                                        recommendations[kind][:topk]                 (app.py:122-144)

What differs, because the reference's file cannot run as written:
  * it has unresolved merge-conflict markers (app.py:38-42, 147-159); the start-up wait here
    is the HEAD side's 120 s;
  * its /api/recommend/* routes call `.get` on the JSONResponse that api_user returns, which
    raises, so they always answered 500; here they read the parsed JSON;
  * its send() timeout sits after a `break` and never fires; here a reader thread feeds a
    queue and a request that gets no line within `timeout` answers 500;
  * the backend is recommendation-system-pokec_amd/pokec_api_cli (csrc/api_cli.cpp, the
    engine's byte-identical api_cli), not build/api_cli.exe; pyngrok (a public tunnel) is
    not part of this build.
Configuration as the reference: config.yaml next to data/ (load_users, server.host,
server.port); POKEC_API_CLI overrides the backend executable.

    python recommendation-system-pokec_amd/app.py --root DIR      (needs a gfx950 GPU: the CLI opens the engine)
"""
import contextlib
import json
import os
import queue
import subprocess
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_CLI = os.path.join(HERE, "pokec_api_cli")
KINDS = {"graph": "graph", "collab": "collaborative", "interest": "interest", "clubs": "clubs"}


def load_config(root):
    """config.yaml as the reference reads it (app.py:15-23); absent file = defaults."""
    cfg = {}
    p = os.path.join(root, "config.yaml")
    if os.path.exists(p):
        import yaml
        with open(p, "r", encoding="utf-8") as f:
            cfg = yaml.safe_load(f) or {}
    srv = cfg.get("server", {}) or {}
    return {"load_users": cfg.get("load_users", 100000), "host": srv.get("host", "0.0.0.0"),
            "port": int(srv.get("port", 8000))}


class ApiCli:
    """The api_cli child process (app.py:29-87): started in `root` (the CLI reads data/ and
    config/ relative to its cwd), READY awaited, one command line in, one JSON line out."""

    def __init__(self, cmd, root, ready_timeout=120.0):
        self.p = subprocess.Popen(cmd, cwd=root, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, text=True, bufsize=1)
        self.lines = queue.Queue()
        self.log = []  # the loader's progress lines before READY
        threading.Thread(target=self._pump, args=(self.p.stdout, self.lines), daemon=True).start()
        threading.Thread(target=self._drain, args=(self.p.stderr,), daemon=True).start()
        self.lock = threading.Lock()
        self.owed = 0  # responses of timed-out requests still to arrive (skipped by the next send)
        deadline = time.time() + ready_timeout
        while True:
            line = self._next(deadline - time.time())
            if line is None:
                self.close()
                raise RuntimeError("api_cli did not signal READY: " + " | ".join(self.log[-5:]))
            if line.strip() == "READY":
                break
            self.log.append(line.rstrip("\n"))

    @staticmethod
    def _pump(stream, q):
        for line in stream:
            q.put(line)
        q.put(None)  # EOF

    @staticmethod
    def _drain(stream):
        for _ in stream:
            pass

    def _next(self, timeout):
        try:
            return self.lines.get(timeout=max(timeout, 0.0))
        except queue.Empty:
            return None

    def send(self, cmd, timeout=10.0):
        """One request: the first non-empty output line (app.py:58-77)."""
        with self.lock:
            while self.owed:  # one line per command: drop the late answers first
                line = self._next(timeout)
                if line is None:
                    raise TimeoutError("api_cli still busy with an earlier request")
                if line.strip():
                    self.owed -= 1
            try:
                self.p.stdin.write(cmd.rstrip("\n") + "\n")
                self.p.stdin.flush()
            except Exception as e:
                raise RuntimeError("failed write to api_cli: " + str(e))
            deadline = time.time() + timeout
            while True:
                line = self._next(deadline - time.time())
                if line is None:
                    if self.p.poll() is not None:
                        raise RuntimeError("api_cli closed output")
                    self.owed += 1
                    raise TimeoutError("timeout waiting for api_cli response")
                if line.strip():
                    return line.strip()

    def close(self):
        try:
            if self.p.poll() is None:
                self.p.stdin.write("EXIT\n")
                self.p.stdin.flush()
                self.p.wait(timeout=5)
        except Exception:
            pass
        if self.p.poll() is None:
            self.p.kill()
            self.p.wait()


def create_app(root, cli_cmd=None, load_users=None, ready_timeout=120.0, request_timeout=10.0):
    """The FastAPI app over an api_cli started in `root`.  cli_cmd: argv of the backend
    (default: pokec_api_cli [load_users], as app.py:31 builds it)."""
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import HTMLResponse, JSONResponse

    cfg = load_config(root)
    n = cfg["load_users"] if load_users is None else load_users
    if cli_cmd is None:
        exe = os.environ.get("POKEC_API_CLI", DEFAULT_CLI)
        if not os.path.exists(exe):
            raise RuntimeError(f"api_cli not found at {exe}. Build it first (make -C recommendation-system-pokec_amd).")
        cli_cmd = [exe, str(int(n))] if n else [exe]
    cli = ApiCli(cli_cmd, root, ready_timeout)

    @contextlib.asynccontextmanager
    async def lifespan(_app):  # the reference's shutdown hook (app.py:96-98)
        yield
        cli.close()

    app = FastAPI(title="Pokec Recommender API (MI355X engine backend)", lifespan=lifespan)
    app.state.cli = cli
    app.state.load_users = n

    @app.get("/", response_class=HTMLResponse)
    async def index():
        return ("<!doctype html><html><head><title>Pokec recommender</title></head><body>"
                f"<h1>Pokec recommender</h1><p>Loaded users: {n}</p>"
                "<p>GET /api/user/{uid}, /api/recommend/{graph|collab|interest|clubs}/{uid}?topk=20</p>"
                "</body></html>")

    @app.get("/health")
    async def health():
        return {"status": "ok", "load_users": n}

    def user_json(uid):
        try:
            out = cli.send(f"USER {uid}", request_timeout)
        except Exception as e:
            raise HTTPException(status_code=500, detail=str(e))
        try:
            return json.loads(out)
        except Exception as e:
            raise HTTPException(status_code=500, detail="invalid JSON from backend: " + str(e) + " output: " + out)

    # plain `def` routes: FastAPI runs them in its threadpool, so a request blocked on the
    # backend (cli.send waits up to request_timeout) never stalls the event loop (/health etc.)
    @app.get("/api/user/{uid}")
    def api_user(uid: int):
        return JSONResponse(user_json(uid))

    def recommend(kind):
        def route(uid: int, topk: int = 20):
            return user_json(uid).get("recommendations", {}).get(KINDS[kind], [])[:topk]
        route.__name__ = f"api_recommend_{kind}"
        return route

    for kind in KINDS:
        app.get(f"/api/recommend/{kind}/{{uid}}")(recommend(kind))
    return app


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=os.getcwd(), help="directory holding data/, config/ and config.yaml")
    args = ap.parse_args()
    cfg = load_config(args.root)
    app = create_app(args.root)
    import uvicorn
    print("Server starting: FastAPI wrapper (MI355X engine backend). Loaded users:", app.state.load_users)
    uvicorn.run(app, host=cfg["host"], port=cfg["port"], log_level="info")


if __name__ == "__main__":
    sys.exit(main())
