"""Model-zoo entry points named like the reference's examples.

The reference's example ElasticJob runs ``python -m model_zoo.iris.dnn_estimator``
(docs/design/elastic-training-operator.md:35 in the reference); this package makes
that command line work unchanged under ``edl submit``.
"""
