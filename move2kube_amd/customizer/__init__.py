"""IR customizers, applied in a fixed order (reference ``internal/customizer/``):
registry (QA; image refs + ``~/.docker/config.json``) -> storage (QA; hostPath to
PVC, storage classes) -> ingress host/TLS (QA)."""

import os

from .. import qaengine
from ..models import ir as irtypes
from ..models import qa
from ..utils import common, fastjson, log, trace
from ..utils.constants import DEFAULT_PVC_SIZE, DEFAULT_REGISTRY_URL, IMAGE_PULL_SECRET_PREFIX, settings

OTHER_REGISTRY = "Other"
ALL_OPTION = "Apply for all"


def _docker_config_dir():
    return os.environ.get("DOCKER_CONFIG") or os.path.join(os.path.expanduser("~"), ".docker")


def _decode_auth(auth):
    """docker/cli ``decodeAuth``: base64 of ``user:password``; ValueError when
    it is not (the whole config file then fails to load)."""
    import base64
    import binascii
    if not auth:
        return
    try:
        decoded = base64.b64decode(auth.replace("\r", "").replace("\n", ""), validate=True)
    except (binascii.Error, ValueError):
        raise ValueError("illegal base64 data")
    if b":" not in decoded:
        raise ValueError("Invalid auth configuration file")


def load_docker_auths():
    """{registry: auth} as ``dockercliconfig.Load`` leaves the docker CLI
    config (``config.json``; registrycustomizer.go:70-92).  Its
    ``LoadFromReader`` decodes every ``auth`` into username and password and
    then clears ``Auth``, so in the reference every value is empty: the
    registries are listed, but no docker-config login is ever offered and the
    default registry stays docker.io.  An auth that does not decode fails the
    whole load (nothing listed).  ``M2K_COMPAT=fixed`` keeps the auths, so the
    "Docker login from config" answer works."""
    path = os.path.join(_docker_config_dir(), "config.json")
    try:
        with open(path) as f:
            cfg = fastjson.load(f)
    except (OSError, ValueError):
        return {}
    auths = {}
    for k, v in ((cfg.get("auths") if isinstance(cfg, dict) else None) or {}).items():
        auth = (v or {}).get("auth", "") if isinstance(v, dict) else ""
        try:
            _decode_auth(auth)
        except ValueError:
            return {}
        auths[k] = auth if settings.fixed else ""
    return auths


def _url_host(regurl):
    """``url.Parse(regurl).Host`` (userinfo dropped, port kept); None on a
    parse error."""
    import urllib.parse
    try:
        netloc = urllib.parse.urlparse(regurl).netloc
    except ValueError:
        return None
    return netloc.rpartition("@")[2]


class RegistryCustomizer:
    def customize(self, ir):
        used = []
        reg_list = [OTHER_REGISTRY]
        newimages = []
        for c in ir.containers:
            if c.new:
                newimages.extend(c.image_names)
        new_folded = {common.go_fold(x) for x in newimages}   # is_string_present, once per image
        for s in ir.sorted_services():
            for c in s.containers:
                if common.go_fold(c.get("image", "")) not in new_folded:
                    parts = c.get("image", "").split("/")
                    if len(parts) == 3:
                        reg_list.append(parts[0])
                        used.append(parts[0])
        auths = {}
        defreg = ""
        if not settings.ignore_environment:
            config_auths = load_docker_auths()
            for regurl in sorted(config_auths):   # a Go map: any order (DEVIATIONS 1)
                auth = config_auths[regurl]
                host = _url_host(regurl)
                if host:
                    regurl = host
                if regurl == "":
                    continue
                if not common.is_string_present(reg_list, regurl):
                    reg_list.append(regurl)
                if auth:
                    defreg = regurl
                    auths[regurl] = auth
        if ir.kubernetes.registry_url == "" and newimages:
            if not common.is_string_present(reg_list, DEFAULT_REGISTRY_URL):
                reg_list.append(DEFAULT_REGISTRY_URL)
            if defreg == "":
                defreg = DEFAULT_REGISTRY_URL
            prob = qa.new_select_problem("Select the registry where your images are hosted:",
                                         ["You can always change it later by changing the yamls."], defreg, reg_list)
            reg = qaengine.fetch_answer(prob).get_string_answer()
            if reg != OTHER_REGISTRY:
                ir.kubernetes.registry_url = reg
        if ir.kubernetes.registry_url == "" and newimages:
            prob = qa.new_input_problem("Enter the name of the registry : ", ["Ex : " + DEFAULT_REGISTRY_URL],
                                        DEFAULT_REGISTRY_URL)
            reg = qaengine.fetch_answer(prob).get_string_answer()
            ir.kubernetes.registry_url = reg or DEFAULT_REGISTRY_URL
        if ir.kubernetes.registry_namespace == "" and newimages:
            prob = qa.new_input_problem("Enter the namespace where the new images are pushed : ", ["Ex : " + ir.name],
                                        ir.name)
            ns = qaengine.fetch_answer(prob).get_string_answer()
            ir.kubernetes.registry_namespace = ns or ir.name
        if not common.is_string_present(used, ir.kubernetes.registry_url):
            used.append(ir.kubernetes.registry_url)
        pull_secrets = {}
        for registry in used:
            dauth = {"auth": "", "username": "", "password": ""}
            docker_login = "Docker login from config"
            no_auth = "No authentication"
            user_login = "UserName/Password"
            existing = "Use existing pull secret"
            options = [existing, no_auth, user_login]
            # the reference looks the auth up by the target registry
            # and names the secret from an empty map value; "fixed" uses the loop's registry
            lookup = ir.kubernetes.registry_url if not settings.fixed else registry
            if lookup in auths:
                if not settings.fixed:
                    pull_secrets[registry] = IMAGE_PULL_SECRET_PREFIX + common.make_file_name_compliant(
                        pull_secrets.get(registry, ""))
                dauth["auth"] = auths[lookup]
                options.append(docker_login)
            prob = qa.new_select_problem("[%s] What type of container registry login do you want to use?" % registry,
                                         ["Docker login from config mode, will use the default config from your local machine."],
                                         no_auth, options)
            auth = qaengine.fetch_answer(prob).get_string_answer()
            if auth == no_auth:
                dauth["auth"] = ""
            elif auth == existing:
                prob = qa.new_input_problem("[%s] Enter the name of the pull secret : " % registry,
                                            ["The pull secret should exist in the namespace where you will be deploying the application."], "")
                name = qaengine.fetch_answer(prob).get_string_answer()
                if name or not settings.fixed:
                    pull_secrets[registry] = name
            elif auth != docker_login:
                prob = qa.new_input_problem("[%s] Enter the container registry username : " % registry,
                                            ["Enter username for container registry login"], "iamapikey")
                dauth["username"] = qaengine.fetch_answer(prob).get_string_answer()
                prob = qa.new_password_problem("[%s] Enter the container registry password : " % registry,
                                               ["Enter password for container registry login."])
                dauth["password"] = qaengine.fetch_answer(prob).get_string_answer()
            if any(dauth.values()):
                # docker's config writer re-derives "auth" from username:password and drops
                # the plain fields, so a config-file login alone serialises as an empty entry
                entry = {}
                if dauth["username"] or dauth["password"]:
                    import base64
                    entry["auth"] = base64.b64encode(("%s:%s" % (dauth["username"], dauth["password"])).encode()).decode()
                elif settings.fixed and dauth["auth"]:
                    entry["auth"] = dauth["auth"]
                if settings.fixed:
                    # the Secret is keyed by, and named after, the registry it authenticates
                    # to; only now is it referenced from imagePullSecrets
                    secret_name = IMAGE_PULL_SECRET_PREFIX + common.make_file_name_compliant(registry)
                    pull_secrets[registry] = secret_name
                    content = fastjson.go_marshal_indent({"auths": {registry: entry}}, "\t")
                else:
                    secret_name = pull_secrets.get(registry, "")
                    # configfile.SaveToWriter: json.MarshalIndent(configFile, "", "\t")
                    content = fastjson.go_marshal_indent({"auths": {ir.kubernetes.registry_url: entry}}, "\t")
                ir.add_storage(irtypes.Storage(name=secret_name, storage_type=irtypes.PULL_SECRET_KIND,
                                               content={".dockerconfigjson": content}))
        ir.values.registry_namespace = ir.kubernetes.registry_namespace
        ir.values.registry_url = ir.kubernetes.registry_url
        for s in ir.sorted_services():
            for c in s.containers:
                image = c.get("image", "")
                if common.go_fold(image) in new_folded:
                    parts = image.split("/")
                    name, tag = common.get_image_name_and_tag(parts[-1])
                    if ir.kubernetes.registry_url and ir.kubernetes.registry_namespace:
                        image = "%s/%s/%s:%s" % (ir.kubernetes.registry_url, ir.kubernetes.registry_namespace, name, tag)
                    elif ir.kubernetes.registry_namespace:
                        image = "%s/%s:%s" % (ir.kubernetes.registry_namespace, name, tag)
                    else:
                        image = "%s:%s" % (name, tag)
                    c["image"] = image
                parts = image.split("/")
                if len(parts) == 3 and parts[0] in pull_secrets:
                    ps = pull_secrets[parts[0]]
                    ips = s.pod_spec.setdefault("imagePullSecrets", [])
                    if not any(e.get("name") == ps for e in ips):
                        ips.append({"name": ps})
        return None


class StorageCustomizer:
    def customize(self, ir):
        self.ir = ir
        self.convert_host_path_to_pvc()
        if not ir.storages:
            log.debug("Empty storage list. Nothing to customize.")
            return None
        if not ir.target_cluster_spec.storage_classes:
            log.warning("No storage classes available in the cluster")
            raise ValueError("No storage classes available in the cluster")
        claims = self.get_pvcs()
        if not claims:
            log.debug("No service with volumes detected. Storage class configuration not required.")
            return None
        keys = list(claims.keys())
        if len(keys) > 1 and not self.should_configure_separately(keys):
            sc = self.select_storage_class(ir.target_cluster_spec.storage_classes, ALL_OPTION, [])
            if settings.fixed:
                # the reference assigns to a loop copy; "fixed" applies the class
                for st in ir.storages:
                    if st.storage_type == irtypes.PVC_KIND:
                        st.pvc_spec["storageClassName"] = sc
            return None
        for st in ir.storages:
            if st.name in claims:
                st.pvc_spec["storageClassName"] = self.select_storage_class(
                    ir.target_cluster_spec.storage_classes, st.name, claims[st.name])
        return None

    def convert_host_path_to_pvc(self):
        ir = self.ir
        visited = {}
        for s in ir.sorted_services():
            log.debug("Service %s has %d volumes", s.name, len(s.volumes))
            for v in s.volumes:
                hp = v.get("hostPath")
                if hp is None:
                    continue
                path = hp.get("path", "")
                if path not in visited:
                    visited[path] = ""
                    log.debug("Detected host path [%r]", v)
                    if not self.should_host_path_be_retained(path):
                        visited[path] = v.get("name", "")
                        v.pop("hostPath", None)
                        v["persistentVolumeClaim"] = {"claimName": v.get("name", "")}
                        ir.add_storage(irtypes.Storage(name=v.get("name", ""), storage_type=irtypes.PVC_KIND, pvc_spec={
                            "volumeName": v.get("name", ""), "resources": {"requests": {"storage": DEFAULT_PVC_SIZE}}}))
                    else:
                        log.debug("Host path [%s] is retained", path)
                else:
                    v.pop("hostPath", None)
                    v["persistentVolumeClaim"] = {"claimName": visited[path]}

    @staticmethod
    def should_host_path_be_retained(path):
        prob = qa.new_confirm_problem("Do you want to create PVC for host path [%s]?:" % path,
                                      ["Use PVC for persistent storage wherever applicable"], False)
        return not qaengine.fetch_answer(prob).get_bool_answer()

    @staticmethod
    def should_configure_separately(claims):
        from ..utils.gotemplate import go_sprint
        ctx = ["Storage classes have to be configured for below claims:", go_sprint(claims)]
        prob = qa.new_confirm_problem("Do you want to configure different storage classes for each claim?", ctx, False)
        return qaengine.fetch_answer(prob).get_bool_answer()

    @staticmethod
    def select_storage_class(classes, claim, services):
        from ..utils.gotemplate import go_sprint
        if claim == ALL_OPTION:
            desc = "Which storage class to use for all persistent volume claims?"
        else:
            desc = "Which storage class to use for persistent volume claim [%s] used by %s" % (claim, go_sprint(services))
        prob = qa.new_select_problem(desc, ["If you have a custom cluster, you can use collect to get storage classes from it."],
                                     classes[0], classes)
        return qaengine.fetch_answer(prob).get_string_answer()

    def get_pvcs(self):
        out = {}
        for st in self.ir.storages:
            if st.storage_type == irtypes.PVC_KIND:
                svcs = []
                for name in sorted(self.ir.services):
                    if any(v.get("name") == st.name for v in self.ir.services[name].volumes):
                        svcs.append(name)
                out[st.name] = svcs
        return out


class IngressCustomizer:
    def customize(self, ir):
        if any(s.service_rel_path != "" for s in ir.services.values()):
            host, secret = self.configure_host_and_tls(ir.name)
            ir.target_cluster_spec.host = host
            ir.ingress_tls_secret_name = secret
        return None

    @staticmethod
    def configure_host_and_tls(name):
        prob = qa.new_input_problem("Provide the ingress host domain", ["Ingress host domain is part of service URL"],
                                    name + ".com")
        host = name + "." + qaengine.fetch_answer(prob).get_string_answer()
        prob = qa.new_input_problem("Provide the TLS secret for ingress", ["Enter TLS secret name"], "")
        secret = qaengine.fetch_answer(prob).get_string_answer()
        return host, secret


def _go_type(x):
    """``%T`` of the reference's value: ``*customizer.<type>``, the Go type name being
    the class name with its first letter lowered."""
    n = type(x).__name__
    return "*customizer." + n[:1].lower() + n[1:]


def get_customizers():
    return [RegistryCustomizer(), StorageCustomizer(), IngressCustomizer()]


def customize(ir):
    log.info("Begin Customization")
    for c in get_customizers():
        log.debug("[%s] Begin Customization", _go_type(c))
        try:
            with trace.span(type(c).__name__, "customizer"):
                c.customize(ir)
        except Exception as e:  # noqa: BLE001
            if isinstance(e, log.FatalError):
                raise
            log.warning("[%s] Failed : %s", _go_type(c), e)
        else:
            log.debug("[%s] Done", _go_type(c))
    log.info("Customization done")
    return ir
