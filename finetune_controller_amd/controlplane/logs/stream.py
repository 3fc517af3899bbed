"""WebSocket log streaming (C16).

Flow of ``/root/reference/app/utils/stream_logger.py:18-514``: wait (<= 300 s, 10 s polls) until the job
is running or already finished, resolve the master pod, send the historical log of container
``pytorch`` in 100-line chunks (50 ms apart), then follow the live log; nothing is sent before the
first line containing ``LOG_STREAM_SEARCH_STRING`` (``Epoch``).  A follow stream that hits EOF checks
the pod phase and stops once the pod is no longer Running/Pending.

The blocking Kubernetes reads run in worker threads; the live stream is consumed line by line from a
thread-side iterator so the event loop never blocks.
"""
from __future__ import annotations

import asyncio
import logging

from ..context import AppContext
from ..schemas.db import DatabaseStatusEnum

logger = logging.getLogger("ftc.logs")

_END = object()


class LogStreamManager:
    def __init__(self, ctx: AppContext, websocket, job_id: str, full_log: bool, follow: bool,
                 last_lines: int = 100, search_string: str | None = None, max_wait: float = 300.0,
                 poll: float = 10.0, chunk_size: int = 100, chunk_delay: float = 0.05):
        self.ctx, self.ws, self.job_id = ctx, websocket, job_id
        self.full_log, self.follow_log = full_log, follow
        self.last_lines = last_lines if not full_log else 0
        self.pod_name: str | None = None
        self.container_name = "pytorch"
        self.chunk_size, self.chunk_delay = chunk_size, chunk_delay
        self.search_string = search_string
        self.search_string_found = not bool(search_string)
        self.is_connected = True
        self.max_wait, self.poll = max_wait, poll

    async def _get_job_status(self):
        last = None
        for attempt in range(3):  # retry with exponential backoff (reference: tenacity x3)
            try:
                return await self.ctx.store.get_job(self.job_id)
            except Exception as e:
                last = e
                await asyncio.sleep(min(10.0, 4.0 * 2 ** attempt) if attempt else 0.5)
        raise last

    async def _send(self, msg: str):
        if not self.is_connected:
            return
        try:
            await self.ws.send_text(msg)
        except Exception as e:
            logger.info("websocket closed for job %s: %s", self.job_id, e)
            self.is_connected = False

    async def _wait_for_job_start(self) -> bool:
        loop = asyncio.get_running_loop()
        t0 = loop.time()
        while self.is_connected:
            if loop.time() - t0 > self.max_wait:
                await self._send("Error: Timeout waiting for job to start")
                return False
            try:
                job = await self._get_job_status()
            except Exception as e:
                await self._send(f"Error while waiting for job to start: {e}")
                return False
            if not job:
                await self._send("Error: Job not found")
                return False
            if job.status in (DatabaseStatusEnum.failed, DatabaseStatusEnum.completed, DatabaseStatusEnum.error,
                              DatabaseStatusEnum.canceled):
                await self._send(f"Info: Job has already finished with status: {job.status.value}")
                return True
            if job.status == DatabaseStatusEnum.running:
                return True
            await self._send(f"Info: Waiting for job to start (current status: {job.status.value})...")
            await asyncio.sleep(self.poll)
        return False

    def _resolve_pod(self) -> str:
        names = self.ctx.kube.get_job_pod_names(self.job_id, self.ctx.namespace, is_master=True)
        if not names:
            raise ValueError(f"No pod names found for job {self.job_id}")
        return names[0]

    async def _pod_active(self) -> bool:
        try:
            pod = await asyncio.to_thread(self.ctx.kube.read_pod, self.ctx.namespace, self.pod_name)
            return pod.get("status", {}).get("phase") in ("Running", "Pending")
        except Exception:
            return False  # gone (404) or unreadable: stop following

    async def _process_and_send(self, lines: list[str]):
        out = []
        for line in lines:
            if not self.search_string_found:
                if self.search_string and self.search_string in line:
                    self.search_string_found = True
                    out.append(line)
            else:
                out.append(line)
        if out:
            await self._send("\n".join(out))

    async def _stream(self):
        ns, kube = self.ctx.namespace, self.ctx.kube
        if self.full_log:
            await self._send("Info: Fetching all previous logs...")
            try:
                text = await asyncio.to_thread(kube.read_pod_log, ns, self.pod_name, self.container_name)
                lines = text.splitlines()
                for i in range(0, len(lines), self.chunk_size):
                    if not self.is_connected:
                        return
                    await self._process_and_send(lines[i:i + self.chunk_size])
                    await asyncio.sleep(self.chunk_delay)
            except Exception as e:
                await self._send(f"Error fetching historical logs: {e}")
        if not self.is_connected:
            return
        if self.follow_log:
            tail = self.last_lines if (not self.full_log and self.last_lines > 0) else None
            await self._send(f"Info: Fetching last {tail} lines and following live logs..." if tail
                             else "Info: Following live logs...")
            if self.full_log:
                # history already sent: follow from the end only
                try:
                    skip = len((await asyncio.to_thread(kube.read_pod_log, ns, self.pod_name,
                                                        self.container_name)).splitlines())
                except Exception:
                    skip = 0
            else:
                skip = 0
            q: asyncio.Queue = asyncio.Queue(maxsize=1024)
            loop = asyncio.get_running_loop()
            stop = {"flag": False}

            def put(item) -> bool:
                # bounded hand-off that gives up once the consumer has left: a put blocked on a full
                # queue nobody drains any more would pin this thread and the pod's log stream forever
                while not stop["flag"]:
                    try:
                        asyncio.run_coroutine_threadsafe(asyncio.wait_for(q.put(item), 1.0), loop).result()
                        return True
                    except asyncio.TimeoutError:
                        continue
                return False

            def pump():
                try:
                    it = kube.stream_pod_log(ns, self.pod_name, self.container_name, tail)
                    n = 0
                    for raw in it:
                        if stop["flag"]:
                            break
                        n += 1
                        if n <= skip:
                            continue
                        if not put(raw):
                            break
                except Exception as e:
                    put(e)
                finally:
                    put(_END)

            fut = loop.run_in_executor(None, pump)
            try:
                while self.is_connected:
                    item = await q.get()
                    if item is _END:
                        if not await self._pod_active():
                            await self._send("Info: Pod has likely completed execution. Stopping log follow.")
                        break
                    if isinstance(item, Exception):
                        await self._send(f"Warning: Error reading log stream: {item}")
                        continue
                    await self._process_and_send([item.decode("utf-8", errors="replace").rstrip("\n")])
            finally:
                stop["flag"] = True
                fut.cancel()
        elif not self.full_log and self.last_lines > 0:
            await self._send(f"Info: Fetching last {self.last_lines} lines...")
            try:
                text = await asyncio.to_thread(kube.read_pod_log, ns, self.pod_name, self.container_name,
                                               self.last_lines)
                await self._process_and_send(text.splitlines())
            except Exception as e:
                await self._send(f"Error fetching last {self.last_lines} lines: {e}")

    async def run(self):
        try:
            await self._wait_for_job_start()
            try:
                self.pod_name = await asyncio.to_thread(self._resolve_pod)
            except Exception as e:
                await self._send(f"Error: Failed to get pod name: {e}")
                return
            await self._stream()
            await self._send("Info: Log streaming finished.")
        except Exception as e:
            logger.error("log streaming failed for job %s: %s", self.job_id, e, exc_info=True)
            await self._send(f"Error: An unexpected error occurred during log streaming: {e}")
        finally:
            if self.is_connected:
                try:
                    await self.ws.close(code=1000)
                except Exception:
                    pass
            self.is_connected = False
