"""Source translator registry (reference ``internal/source/translator.go``).

Fixed order: Dockerfile, Compose, CfManifest, Knative, Kube, and Any2Kube last.
``translate`` picks ``services[0]`` of every plan service, dispatches it to the
translator of its ``translationType`` and merges the resulting IRs.
"""

from ..models import ir as irtypes
from ..utils import log, trace


class Translator:
    translation_type = ""

    def get_translator_type(self):
        return self.translation_type

    def get_service_options(self, input_path, plan):
        raise NotImplementedError

    def translate(self, services, plan):
        raise NotImplementedError

    def __repr__(self):
        return "*source.%s" % type(self).__name__


def get_source_loaders():
    from .any2kube import Any2KubeTranslator
    from .cfmanifest2kube import CfManifestTranslator
    from .compose2kube import ComposeTranslator
    from .dockerfile2kube import DockerfileTranslator
    from .knative2kube import KnativeTranslator
    from .kube2kube import KubeTranslator
    return [DockerfileTranslator(), ComposeTranslator(), CfManifestTranslator(), KnativeTranslator(),
            KubeTranslator(), Any2KubeTranslator()]


def translate(plan):
    ir = irtypes.new_ir(plan)
    log.info("Begin Translation")
    for t in get_source_loaders():
        log.info("[%r] Begin translation", t)
        valid = []
        for name in sorted(plan.services):
            options = plan.services[name]
            if options and options[0].translation_type == t.get_translator_type():
                valid.append(options[0])
        log.debug("Services to translate : %d", len(valid))
        try:
            with trace.span(type(t).__name__, "translate", services=len(valid)):
                cur = t.translate(valid, plan)
        except Exception as e:  # noqa: BLE001
            # the counts are logged before the error check (translator.go:58-64)
            log.debug("Services translated : %d", 0)
            log.debug("Containers translated : %d", 0)
            log.warning("[%r] Failed : %s", t, e)
            continue
        log.debug("Services translated : %d", len(cur.services))
        log.debug("Containers translated : %d", len(cur.containers))
        log.info("[%r] Done", t)
        ir.merge(cur)
        log.debug("Total Services after translation : %d", len(ir.services))
        log.debug("Total Containers after translation : %d", len(ir.containers))
    log.info("Translation done")
    return ir
