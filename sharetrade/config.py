"""Typed configuration for the sharetrade engine.

The reference hard-codes every algorithmic knob as a Scala constant and keeps
runtime settings in HOCON (`src/main/resources/application.conf:1-25`,
`src/test/resources/application.conf:1-11`).  Here every knob lives in one
dataclass tree with the reference values as the ``reference_compat`` preset
(SURVEY.md §5.6):

=====================  ==========================  =====================================
knob                   reference value             cite
=====================  ==========================  =====================================
actions / order        Buy, Sell, Hold             QDecisionPolicyActor.scala:17
input dim              203 = 201 prices + 2        QDecisionPolicyActor.scala:18
epsilon (max exploit)  0.9                         QDecisionPolicyActor.scala:19
exploit ramp           min(eps, step/1000)         QDecisionPolicyActor.scala:58
gamma                  0.001                       QDecisionPolicyActor.scala:20
hidden                 [200] + ReLU on output      QDecisionPolicyActor.scala:22,47
init                   W~N(0,1), biases 0.1 const  QDecisionPolicyActor.scala:41-46
optimizer              AdaGrad(0.01)               QDecisionPolicyActor.scala:50
snapshot interval      500 updates                 QDecisionPolicyActor.scala:74
rollout workers        10                          TrainerRouterActor.scala:36
backoff                3 s / 60 s / 0.2            TrainerRouterActor.scala:46-51
ask timeouts           20 s app, 10 s router/child ShareTradeHelper.scala:18; ...:42; ...:28
poll                   201 x 5 s, Await 10 s       ShareTradeHelper.scala:32-33,45
budget / shares        2400.0 / 0                  ShareTradeHelper.scala:20-21
progress log every     200 steps                   TrainerChildActor.scala:108
=====================  ==========================  =====================================

Configs load from JSON or TOML files and accept ``a.b.c=value`` CLI overrides.
"""
from __future__ import annotations

import copy
import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

ACTIONS = ("Buy", "Sell", "Hold")  # index order 0,1,2 (QDecisionPolicyActor.scala:17)


@dataclass
class ModelConfig:
    """Q-network architecture (an MLP over the 203-feature trading state)."""

    history: int = 201              # prices per state window (QDecisionPolicyActor.scala:18)
    hidden: List[int] = field(default_factory=lambda: [200])
    n_actions: int = 3
    output_relu: bool = True        # quirk Q3 (QDecisionPolicyActor.scala:47)
    train_bias: bool = False        # quirk Q4: tf.constant biases (QDecisionPolicyActor.scala:42,46)
    bias_init: float = 0.1
    init_std: float = 1.0           # tf.RandomNormalInitializer() default N(0,1)
    init: str = "normal"            # "normal" (reference) | "he" (scaled, for deep nets)
    # weight draws: "philox" (counter-based Philox + Box-Muller: the init_normal HIP kernel on a GPU,
    # its NumPy mirror on the host) | "torch" (torch's CPU generator)
    init_rng: str = "philox"

    @property
    def input_dim(self) -> int:
        return self.history + 2


@dataclass
class AgentConfig:
    """Q-learning hyper-parameters."""

    epsilon: float = 0.9            # max exploit probability
    ramp: float = 1000.0            # exploit prob = min(epsilon, step / ramp)
    gamma: float = 0.001
    optimizer: str = "adagrad"      # adagrad | adam | sgd
    lr: float = 0.01
    adagrad_init_acc: float = 0.1   # TF default initial accumulator (SURVEY §5.6 knob)
    adam_betas: List[float] = field(default_factory=lambda: [0.9, 0.999])
    adam_eps: float = 1e-8
    # "compat": TD target written at argmax(q_next) (quirk Q2, QDecisionPolicyActor.scala:69-71)
    # "action": TD target written at the taken action (the intended semantics)
    target_slot: str = "compat"
    loss_reduction: str = "sum"     # "sum" over the batch (reference, B=1) | "mean"
    # "absolute": reward = change of portfolio value in $ (TrainerChildActor.scala:142-143);
    # "relative": the portfolio's one-step return (change / previous value) -- scale-free across
    # envs whose prices drift apart (bf16 engine kernels and the torch oracle); "growth": that return minus
    # half its square, the portfolio's log growth to second order (Kelly: its expectation peaks at a position
    # of mu / sigma^2 of wealth instead of at the largest one)
    reward_mode: str = "absolute"
    td_clip: float = 0.0            # > 0: clamp the TD error fed back (Huber loss); 0 = squared error
    # learning-quality experiments (tools/learning_eval.py, preset flagship_stable): the torch backend, the
    # native batched fp32 step and the flagship bf16 ws step implement them (the wide / narrow bf16 kernels
    # refuse non-default values):
    target_every: int = 0           # > 0: Q(x') from a target copy of the params, refreshed every N steps
    double_dqn: bool = False        # with target_every: max-Q(x') action by the online net, valued by the target
    reward_scale: float = 1.0       # multiplies the reward in the TD target
    ramp_mode: str = "position"     # exploit ramp over the episode position (reference) | "global": the step count
    snapshot_interval: int = 500    # QDecisionPolicyActor.scala:74
    seed: int = 1234


@dataclass
class EnvConfig:
    """Trading environment."""

    budget: float = 2400.0          # ShareTradeHelper.scala:20
    shares: int = 0                 # ShareTradeHelper.scala:21
    # quirk Q1: decisions use the constructor budget/shares (TrainerChildActor.scala:120-122)
    compat_decisions: bool = True
    # feature normalisation of the state row: "raw" (reference) | "relative"
    features: str = "raw"
    progress_every: int = 200       # TrainerChildActor.scala:108


@dataclass
class DataConfig:
    source: str = "csv"             # csv | linear | random_walk | ar1 (one-day momentum) | trend (persistent drift)
    ticker: str = "MSFT"
    start: str = "1992-01-01"
    end: str = "2015-01-01"
    filter_range: bool = False      # quirk Q10: reference ignores the date range
    csv_path: Optional[str] = None  # default: config.default_csv_path() (env var, reference CSV, bundled series)
    length: int = 6047              # synthetic series length
    start_price: float = 50.0
    volatility: float = 0.02
    ar_phi: float = 0.3             # ar1 source: log-return autocorrelation
    # trend source: log-return = mu_t + volatility * eps_t with a persistent, zero-mean drift
    # mu_t = rho mu_{t-1} + trend_sd sqrt(1 - rho^2) eta_t (regimes lasting ~1 / (1 - rho) days): a signal
    # that a policy moving one share per step can follow, unlike ar1's one-day momentum
    # synthetic banks (random_walk, ar1, trend) generated on a 16-bit tick grid per series (price = tick * 2^x,
    # tick <= 65535: a tick is <= 2^-16 of the series' largest price): the flagship kernel then streams its
    # windows as u16 ticks with bit-identical features (data.prices.tick16_quantize, csrc/series.hip tick16)
    tick16: bool = True
    trend_rho: float = 0.995
    trend_sd: float = 0.002
    seed: int = 7


@dataclass
class RouterConfig:
    n_workers: int = 10             # TrainerRouterActor.scala:36
    backoff_min_s: float = 3.0      # TrainerRouterActor.scala:48
    backoff_max_s: float = 60.0     # TrainerRouterActor.scala:49
    backoff_jitter: float = 0.2     # TrainerRouterActor.scala:50
    ask_timeout_s: float = 10.0     # TrainerRouterActor.scala:42, TrainerChildActor.scala:28
    app_ask_timeout_s: float = 20.0  # ShareTradeHelper.scala:18
    poll_interval_s: float = 5.0    # ShareTradeHelper.scala:33
    poll_rounds: int = 201          # ShareTradeHelper.scala:32
    await_s: float = 10.0           # ShareTradeHelper.scala:45
    reply_result: bool = True       # quirk Q9 fixed: GetAvg/GetStd reply Result(x)
    redispatch_on_restart: bool = True  # quirk Q14 fixed


@dataclass
class PersistConfig:
    """Akka persistence settings (application.conf:5-18)."""

    journal_plugin: str = "file"    # file (native C++ journal) | inmemory (test profile)
    journal_dir: str = "target/my/journal"
    snapshot_dir: str = "target/my/snapshots"
    persist_before_reply: bool = False  # quirk Q11: reference replies before persisting
    merge_on_recovery: bool = True      # quirk Q10 fixed: merge tickers on recovery


@dataclass
class EngineConfig:
    """GPU vectorized engine (data plane)."""

    device: str = "auto"            # auto | cuda | cpu
    envs_per_rank: int = 10
    dtype: str = "bf16"             # bf16 (MFMA fused step) | fp32 (exact path)
    # envs per LDS chunk of the fused bf16 step kernel: 0 = auto (64 when E % 64 == 0, else 32);
    # 64 = csrc/qstep_wide.hip (layer-1 weights in VGPRs), 32 = csrc/qstep_fused.hip (weights in LDS)
    chunk: int = 0
    step_waves: int = 8             # 64-env-chunk kernel: 8 waves (two per SIMD, measured fastest) or 4
    # fused bf16 step kernel: "auto" (ws where its geometry fits, else by chunk), "ws" (csrc/qstep_ws.hip:
    # wave-specialised, data waves run whole 16-env tiles, gradient waves consume them through an LDS ring;
    # E % 64 == 0, history 201, dims 224-128-128, static schedule), "wide" (csrc/qstep_wide.hip, 64-env
    # chunks) or "narrow" (csrc/qstep_fused.hip, 32-env chunks)
    step_kernel: str = "auto"
    # fp32 engine (engine.dtype = "fp32": the reference geometry): "auto" = the batched MFMA step
    # (csrc/mlp_f32_mfma.hip) from 1,024 envs up, the per-env row kernels (csrc/mlp_f32.hip) below; "on" / "off"
    f32_batched: str = "auto"
    # batched fp32 step: weight-gradient split-K partials + bias column sums added in a fixed order instead of
    # fp32 atomics (bit-reproducible); "auto" = on for DP ranks and env.compat_decisions (reference_compat)
    f32_deterministic: str = "auto"
    step_variant: str = ""          # timing / debug build of the ws kernel (csrc/ab/qstep_ws_<v>.hip); opt-in only
                                    # (SHARETRADE_AB_BUILDS=1, several compute wrong results); "" = production
    graph: bool = True              # capture the step in a HIP graph
    graph_steps: int = 16           # steps per graph replay in VectorEngine.run (fewer launch boundaries)
    backend: str = "auto"           # auto | native | torch
    bucket_mb: float = 4.0          # DP gradient all-reduce bucket (one call below this size)
    grad_compress: str = ""         # "" | "bf16" (wire format of the DP all-reduce)
    slab_dtype: str = "bf16"        # per-workgroup gradient partials of the 64-env-chunk kernel: "bf16" | "fp32"
    # DP gradient all-reduce overlapped with the next step's fused kernel: the gradient of step t
    # is applied after step t+1's kernel (one-step delay, identical on every rank).  The reference
    # applies updates asynchronously through one mailbox; False = strict sync DP (bit-equal to one
    # process holding all envs).
    dp_overlap: bool = False
    # chunk schedule of the 64-env-chunk step kernel: "static" (chunk k of workgroup i = i + k*grid,
    # bit-reproducible), "dynamic" (per-XCD claim heads: workgroups whose CU is still held by the
    # overlapped RCCL all-reduce take fewer chunks instead of stretching the launch), or "auto"
    # (dynamic for the wide kernel under overlapped DP with world_size > 1, else static: the ws kernel's
    # dynamic build is 14 % slower, profiles/r4_flagship_dp.md)
    chunk_schedule: str = "auto"
    # ws step kernel + relative features: read the price windows from a 16-bit tick copy of the bank when every
    # series is exactly on a tick grid (data.tick16, or user data that is): "auto" | "off" (the fp32 windows)
    bank16: str = "auto"
    grid: int = 0                   # step-kernel workgroups: 0 = one per CU (capped at the chunk count)
    # > 0: keep a Polyak (exponential moving) average of the parameters, updated by the optimizer pass
    # after every step: ema <- ema + (1 - ema_decay) (w - ema).  The averaged weights are the ones to
    # serve (VectorEngine.serving_params; a single online-DQN snapshot's greedy policy drifts between
    # steps, profiles/r2_serve_eval.md)
    ema_decay: float = 0.0


@dataclass
class LogConfig:
    loglevel: str = "INFO"          # application.conf:3
    test_listener: bool = False     # src/test/resources/application.conf:5


@dataclass
class Config:
    model: ModelConfig = field(default_factory=ModelConfig)
    agent: AgentConfig = field(default_factory=AgentConfig)
    env: EnvConfig = field(default_factory=EnvConfig)
    data: DataConfig = field(default_factory=DataConfig)
    router: RouterConfig = field(default_factory=RouterConfig)
    persist: PersistConfig = field(default_factory=PersistConfig)
    engine: EngineConfig = field(default_factory=EngineConfig)
    log: LogConfig = field(default_factory=LogConfig)

    # ------------------------------------------------------------------ io
    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), indent=2, sort_keys=True)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Config":
        cfg = cls()
        _merge(cfg, d)
        return cfg

    @classmethod
    def load(cls, path: str, preset: str = "reference_compat") -> "Config":
        cfg = preset_config(preset)
        with open(path, "rb") as f:
            raw = f.read()
        if path.endswith(".toml"):
            import tomli

            d = tomli.loads(raw.decode())
        elif path.endswith(".conf") or path.endswith(".hocon"):
            # Akka-style application.conf (the reference's configuration format)
            from .utils import hocon

            d, _ = hocon.akka_to_config(hocon.loads(raw.decode()))
        else:
            d = json.loads(raw.decode())
        _merge(cfg, d)
        return cfg

    def override(self, items: Sequence[str]) -> "Config":
        """Apply ``section.key=value`` overrides (values parsed as JSON when possible)."""
        for it in items:
            if "=" not in it:
                raise ValueError(f"override must be key=value: {it!r}")
            key, val = it.split("=", 1)
            try:
                v: Any = json.loads(val)
            except json.JSONDecodeError:
                v = val
            node: Any = self
            parts = key.split(".")
            for p in parts[:-1]:
                node = getattr(node, p)
            if not hasattr(node, parts[-1]):
                raise KeyError(f"unknown config key {key}")
            setattr(node, parts[-1], v)
        return self

    def clone(self) -> "Config":
        return copy.deepcopy(self)


def _merge(obj: Any, d: Dict[str, Any]) -> None:
    for k, v in d.items():
        if not hasattr(obj, k):
            raise KeyError(f"unknown config key {k}")
        cur = getattr(obj, k)
        if dataclasses.is_dataclass(cur) and isinstance(v, dict):
            _merge(cur, v)
        else:
            setattr(obj, k, v)


def preset_config(name: str = "reference_compat") -> Config:
    """Named presets.

    * ``reference_compat`` — the reference's constants and quirks.
    * ``intended`` — same network but with the quirks fixed (default semantics).
    * ``flagship`` — BASELINE.json config 2/3: 2x128 MLP, bf16 fused step,
      normalised features, correct env/TD semantics, Adam.
    * ``flagship_stable`` — ``flagship`` plus the learning stabilisers that make its greedy policy beat
      buy-and-hold's median on the AR(1) and trend banks (profiles/r5_learning_ws_knobs*.md): a target
      network refreshed every 1,000 steps, Double DQN, reward scale 100, the exploit ramp over 3,000
      training steps, gamma 0.99.  Same fused bf16 step (its knob build + csrc/qtarget.hip), ~1.7x its time.
    * ``test`` — the test profile (src/test/resources/application.conf): in-memory
      journal, DEBUG log level, test event listener.
    """
    cfg = Config()
    if name == "reference_compat":
        cfg.engine.dtype = "fp32"
        return cfg
    if name == "intended":
        cfg.engine.dtype = "fp32"
        cfg.env.compat_decisions = False
        cfg.agent.target_slot = "action"
        cfg.model.output_relu = False
        cfg.model.train_bias = True
        return cfg
    if name == "flagship":
        cfg.model.hidden = [128, 128]
        cfg.model.output_relu = False
        cfg.model.train_bias = True
        cfg.model.init = "he"
        cfg.env.compat_decisions = False
        cfg.env.features = "relative"
        cfg.agent.target_slot = "action"
        cfg.agent.optimizer = "adam"
        cfg.agent.lr = 1e-3
        cfg.agent.loss_reduction = "mean"
        cfg.agent.gamma = 0.9            # tools/learning_curve.py: stable and learns (0.99 drifts)
        cfg.agent.reward_mode = "relative"
        cfg.data.source = "random_walk"
        cfg.engine.dtype = "bf16"
        cfg.engine.envs_per_rank = 65536
        return cfg
    if name == "flagship_stable":
        cfg = preset_config("flagship")
        a = cfg.agent
        a.target_every, a.double_dqn, a.reward_scale = 1000, True, 100.0
        a.ramp_mode, a.ramp, a.gamma = "global", 3000.0, 0.99
        return cfg
    if name == "recurrent":
        # BASELINE config 5: GRU(256) Q-net on minute bars (sharetrade/trainer/recurrent.py)
        cfg = preset_config("flagship")
        cfg.agent.lr = 3e-4
        cfg.data.source = "minute_bars"
        return cfg
    if name == "test":
        cfg.engine.dtype = "fp32"
        cfg.persist.journal_plugin = "inmemory"
        cfg.log.loglevel = "DEBUG"
        cfg.log.test_listener = True
        return cfg
    raise KeyError(f"unknown preset {name}")


REFERENCE_CSV = "/root/reference/src/main/resources/MSFT-stock-prices-revised.txt"
BUNDLED_SERIES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "msft_prices.npz")


def default_csv_path() -> str:
    """Where the MSFT daily series comes from (the reference bundles it as a classpath resource,
    `SharePriceGetter.scala:90`).  Resolution order -- documented, and reported by
    :func:`price_data_origin`:

    1. ``SHARETRADE_MSFT_CSV`` (any ``price, yyyy-MM-dd`` file, or a ``.npz`` series);
    2. the reference checkout's CSV, when present (parsed in place);
    3. ``sharetrade/data/msft_prices.npz``: the same series, parsed once from the reference CSV
       (``tools/make_msft_fixture.py``; ``tests/test_app.py`` re-checks it against the CSV whenever the
       CSV exists), so parity runs work on machines without the reference checkout (the GPU boxes).
    """
    env = os.environ.get("SHARETRADE_MSFT_CSV")
    if env:
        return env
    if os.path.exists(REFERENCE_CSV):
        return REFERENCE_CSV
    return BUNDLED_SERIES


def price_data_origin() -> str:
    p = default_csv_path()
    return "bundled" if p == BUNDLED_SERIES else ("env" if os.environ.get("SHARETRADE_MSFT_CSV") else "reference")
