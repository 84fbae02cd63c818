__all__ = ["define_estimator", "define_losses", "define_optimizer", "define_metrics"]
