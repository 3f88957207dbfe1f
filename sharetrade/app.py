"""``ShareTradeHelper`` — the application driver (`ShareTradeHelper.scala:14-48`).

Reference flow: create the ActorSystem, the policy actor, the price getter
and the router (budget 2400.0, 0 shares); ask for MSFT 1992-01-01..2015-01-01;
pipe ``SendTrainingData`` to the router; ``StartTraining``; then poll up to
201 times every 5 s with three parallel asks (``IsEverythingDone``, ``GetAvg``,
``GetStd``) until ``(Completed, Result(avg), Result(std))`` and log them.

Fixed here: the router replies ``Result`` (quirk Q9 — the reference's App could
never match its router's bare ``Double``), and the system is shut down with an
exit status when done or when polling gives up (Q12).

Two training back ends behind the same actors and messages:

* ``engine="actors"`` — every worker runs the reference's per-step
  ``SelectionAction`` / ``UpdateQ`` protocol against the shared
  ``QDecisionPolicyActor`` (fp32, batch-1 semantics);
* ``engine="vector"`` — the workers are lanes of one :class:`VectorEngine`
  driven by an ``EngineActor`` (fused HIP step kernel on a GPU): same message
  API, same lifecycle, orders of magnitude more env-steps/s.
"""
from __future__ import annotations

import logging
import time
from typing import Dict, Optional

import torch

from .actors.runtime import ActorSystem, pipe_to
from .config import Config, preset_config
from .data.getter import SharePriceGetter
from .data.prices import to_date
from .policy.actor import QDecisionPolicyActor
from .protocol import (Completed, GetAvg, GetStd, IsEverythingDone, RequestStockPrice, Result, SendTrainingData,
                       StartTraining)
from .trainer.router import TrainerRouterActor

logger = logging.getLogger("sharetrade.ShareTradeHelper")


def run(cfg: Optional[Config] = None, engine: str = "actors", device: Optional[str] = None,
        max_prices: Optional[int] = None, quiet: bool = False, gpus: int = 1,
        dp: Optional[Dict] = None) -> Dict[str, float]:
    """Run the application; returns ``{"avg", "std", "completed", "elapsed_s", ...}``.

    ``engine="vector", gpus=N > 1``: the router's N routees are the ranks of a data-parallel group, one
    process per GPU (``sharetrade/trainer/dp_actors.py``); ``dp`` passes the group's options
    (``device`` "cuda" / "cpu", ``backend``, ``envs_per_rank``, ``ckpt_dir``, ``ckpt_every``,
    ``same_device``, ``out_dir``, ``group_kw``).  The parent process never touches the GPU."""
    cfg = cfg or preset_config("reference_compat")
    rc = cfg.router
    dp_mode = engine == "vector" and int(gpus) > 1
    dev = None if dp_mode else _device(device or cfg.engine.device)
    system = ActorSystem("ShareTradeHelperSystem", loglevel=cfg.log.loglevel)
    t0 = time.perf_counter()
    out: Dict[str, float] = {"completed": 0.0}
    try:
        budget, shares = cfg.env.budget, cfg.env.shares
        request = RequestStockPrice(cfg.data.ticker, to_date(cfg.data.start), to_date(cfg.data.end))
        policy = system.actor_of(QDecisionPolicyActor.props(cfg, device=dev if engine == "actors" else None),
                                 "Q-policy-actor")
        getter = system.actor_of(SharePriceGetter.props(cfg=cfg), "Share-price-getter-actor")
        prices = getter.ask(request, rc.app_ask_timeout_s)
        if max_prices:
            from .protocol import StockDataResponse, TreeMap

            prices = prices.map(lambda r: StockDataResponse(r.stock_name,
                                                            TreeMap(list(r.share_prices.items())[:max_prices])))
        if dp_mode:
            from .actors.runtime import Props
            from .trainer.dp_actors import DPRouterActor, RankGroupActor, rank_routee_props

            o = dict(dp or {})
            o.setdefault("device", "cuda" if (device or "cuda").startswith("cuda") else "cpu")
            group = system.actor_of(RankGroupActor.props(cfg, int(gpus), **o), "Rank-group-actor")
            router = system.actor_of(Props(DPRouterActor, group, policy, budget, shares, cfg,
                                           child_trainer_props=rank_routee_props(group, cfg), n_children=int(gpus)),
                                     "Trainer-parent-actor")
            out["dp_group"] = group
        elif engine == "vector":
            from .trainer.engine_actor import EngineActor, engine_child_props

            eng = system.actor_of(EngineActor.props(cfg, device=dev), "Engine-actor")
            router = system.actor_of(TrainerRouterActor.props(policy, budget, shares, cfg,
                                                              child_trainer_props=engine_child_props(eng, cfg)),
                                     "Trainer-parent-actor")
        else:
            router = system.actor_of(TrainerRouterActor.props(policy, budget, shares, cfg), "Trainer-parent-actor")
        pipe_to(prices.map(SendTrainingData), router)
        router.tell(StartTraining)
        for _ in range(rc.poll_rounds):
            time.sleep(rc.poll_interval_s)
            fc = router.ask(IsEverythingDone, rc.app_ask_timeout_s)
            fa = router.ask(GetAvg, rc.app_ask_timeout_s)
            fs = router.ask(GetStd, rc.app_ask_timeout_s)
            try:
                c, a, s = fc.result(rc.await_s), fa.result(rc.await_s), fs.result(rc.await_s)
            except Exception as e:  # noqa: BLE001 - the reference's Await would throw here
                logger.debug("poll failed: %r", e)
                continue
            if c is Completed and isinstance(a, Result) and isinstance(s, Result):
                if not quiet:
                    logger.info("avg is %s, std is %s", a.double, s.double)
                out.update(avg=a.double, std=s.double, completed=1.0)
                break
        grp = out.pop("dp_group", None)
        if grp is not None:
            # per-rank episode records and the ranks' deaths / generations (tests, CLI report)
            try:
                out["dp"] = grp.ask(_DPInfo, 10.0).result(10.0)
            except Exception:  # noqa: BLE001 - the report is best effort
                pass
    finally:
        out.pop("dp_group", None)
        out["elapsed_s"] = time.perf_counter() - t0
        system.terminate()
    return out


from .trainer.dp_actors import GetDPInfo as _DPInfo  # noqa: E402


def _device(spec: Optional[str]) -> torch.device:
    if spec in (None, "auto"):
        return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(spec)
