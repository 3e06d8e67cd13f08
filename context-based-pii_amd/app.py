"""Flask drop-in for main_service's three hot-path endpoints, with request
micro-batching in front of the engine.

Routes, request and response JSON are those of the reference (main_service/main.py):

* ``POST /handle-agent-utterance``     {conversation_id, transcript} -> {redacted_transcript, context_stored}   (:344-384)
* ``POST /handle-customer-utterance``  {conversation_id, transcript} -> {redacted_transcript, context_used}     (:386-425)
* ``POST /redact-utterance-realtime``  {conversation_id, utterance}  -> {redacted_utterance}                    (:427-466)

The reference serves them from gunicorn with 8 threads (main_service/Dockerfile:29), one blocking
DLP RPC per request.  Here every request thread hands its request to a :class:`MicroBatcher`; one
dispatcher thread drains whatever requests are waiting (up to ``max_batch``, waiting at most
``max_wait_s`` for more once one has arrived) and runs them through
``PiiService.process_requests`` -- one engine call per micro-batch, results identical to serving the
requests one by one in arrival order.  Authentication (``@firebase_auth_required`` on the realtime
route, main.py:428) is deployment glue and out of scope; the shim accepts every request.

    python -m context-based-pii_amd.app  (or create_app() under any WSGI server)
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import List, Optional, Tuple

from .service import PartialBatchError, PiiService


class MicroBatcher:
    """Coalesces concurrent handler requests into one engine call each."""

    def __init__(self, service, max_batch: int = 1024, max_wait_s: float = 0.001):
        self.service = service
        self.max_batch = max_batch
        self.max_wait_s = max_wait_s
        self.q: "queue.Queue" = queue.Queue()
        self.batches: List[int] = []           # sizes of the micro-batches run (observability)
        self._thread = threading.Thread(target=self._loop, name="pii-microbatcher", daemon=True)
        self._thread.start()

    def submit(self, kind: str, data: Optional[dict]) -> Tuple[dict, int]:
        f: Future = Future()
        self.q.put((kind, data, f))
        return f.result()

    def close(self) -> None:
        self.q.put(None)
        self._thread.join(timeout=5)

    def _loop(self) -> None:
        while True:
            item = self.q.get()
            if item is None:
                return
            batch = [item]
            deadline = time.monotonic() + self.max_wait_s
            stop = False
            while len(batch) < self.max_batch:
                try:
                    nxt = self.q.get_nowait()
                except queue.Empty:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        break
                    try:
                        nxt = self.q.get(timeout=left)
                    except queue.Empty:
                        break
                if nxt is None:
                    stop = True
                    break
                batch.append(nxt)
            self.batches.append(len(batch))
            try:
                res = self.service.process_requests([(k, d) for k, d, _ in batch])
                for (_, _, f), r in zip(batch, res):
                    f.set_result(r)
            except Exception as exc:
                # a failure that request validation did not foresee: the requests whose sub-batch
                # completed keep their responses (their context is committed: running them again
                # would store it twice); the rest run one at a time, so that only the request that
                # raises fails (as it would alone in the reference's per-request handler), and no
                # request thread is left waiting
                done = exc.done if isinstance(exc, PartialBatchError) else {}
                for i, (_, _, f) in enumerate(batch):
                    if i in done and not f.done():
                        f.set_result(done[i])
                for k, d, f in batch:
                    if f.done():
                        continue
                    try:
                        f.set_result(self.service.process_requests([(k, d)])[0])
                    except Exception as e:
                        f.set_exception(e)
            if stop:
                return


def create_app(service: Optional[PiiService] = None, max_batch: int = 1024, max_wait_s: float = 0.001):
    from flask import Flask, jsonify, request

    svc = service if service is not None else PiiService()
    app = Flask("context-based-pii_amd")
    batcher = MicroBatcher(svc, max_batch=max_batch, max_wait_s=max_wait_s)
    app.config["PII_SERVICE"] = svc
    app.config["PII_BATCHER"] = batcher

    def serve(kind):
        body, status = batcher.submit(kind, request.get_json(silent=True))
        return jsonify(body), status

    @app.route("/handle-agent-utterance", methods=["POST"])
    def handle_agent_utterance():
        return serve("agent")

    @app.route("/handle-customer-utterance", methods=["POST"])
    def handle_customer_utterance():
        return serve("customer")

    @app.route("/redact-utterance-realtime", methods=["POST"])
    def redact_utterance_realtime():
        return serve("realtime")

    return app


if __name__ == "__main__":      # pragma: no cover - manual serving
    import os
    create_app().run(host="127.0.0.1", port=int(os.environ.get("PORT", "8080")), threaded=True)
