"""Exception types named after the JVM exceptions the reference's supervision
strategy maps to directives (`TrainerRouterActor.scala:53-58`)."""


class IllegalArgumentException(ValueError):
    """Bad input shape / too few prices (`QDecisionPolicyActor.scala:56-57,64-65`,
    `TrainerChildActor.scala:69-70`) -> supervision directive Stop."""


class ArithmeticException(ArithmeticError):
    """-> Resume."""


class NullPointerException(Exception):
    """-> Restart (with backoff)."""
