"""The intermediate representation (reference ``internal/types/ir.go:36-409``).

A service carries a Kubernetes ``PodSpec`` in its JSON form (camelCase keys,
exactly what ends up in the manifests); containers describe images to build
or reuse; storages describe PVCs/ConfigMaps/Secrets/pull secrets.

Merge semantics are the reference's: services are replaced by name (with a
warning), containers merge when they share an image name *and* build type,
storages merge by name.  Go map iteration order is random in the reference;
here every consumer iterates services in sorted-name order (determinism fix,
documented in SURVEY.md section 7.4 #5).
"""


from ..utils import common, log
from ..utils.constants import ANNOTATION_LABEL_VALUE
from . import plan as plantypes
from .collection import ClusterMetadataSpec
from .output import HelmValues

SECRET_KIND = "Secret"
CONFIGMAP_KIND = "ConfigMap"
PVC_KIND = "PersistentVolumeClaim"
PULL_SECRET_KIND = "PullSecret"


class Port:
    """networkingv1.ServiceBackendPort: a port number with an optional name."""
    __slots__ = ("name", "number")

    def __init__(self, number=0, name=""):
        self.name = name
        self.number = number

    def __eq__(self, o):
        return isinstance(o, Port) and self.name == o.name and self.number == o.number

    def __repr__(self):
        return "Port(%r, %r)" % (self.number, self.name)


class PortForwarding:
    __slots__ = ("service_port", "pod_port")

    def __init__(self, service_port, pod_port):
        self.service_port = service_port
        self.pod_port = pod_port

    def __eq__(self, o):
        return isinstance(o, PortForwarding) and self.service_port == o.service_port and self.pod_port == o.pod_port

    def __repr__(self):
        return "PortForwarding(%r -> %r)" % (self.service_port, self.pod_port)


class Service:
    def __init__(self, name="", service_rel_path=""):
        self.pod_spec = {}
        self.name = name
        self.backend_service_name = ""
        self.annotations = None
        self.labels = None
        self.port_forwardings = []
        self.replicas = 0
        self.networks = []
        self.service_rel_path = service_rel_path
        self.only_ingress = False
        self.daemon = False

    # PodSpec conveniences
    @property
    def containers(self):
        # reading leaves pod_spec as it was (a Go range over a nil slice does
        # not allocate one); assign through the setter to add containers
        cs = self.pod_spec.get("containers")
        return cs if cs is not None else []

    @containers.setter
    def containers(self, v):
        self.pod_spec["containers"] = v

    @property
    def volumes(self):
        return self.pod_spec.get("volumes") or []

    @volumes.setter
    def volumes(self, v):
        self.pod_spec["volumes"] = v

    @property
    def restart_policy(self):
        return self.pod_spec.get("restartPolicy", "")

    @restart_policy.setter
    def restart_policy(self, v):
        self.pod_spec["restartPolicy"] = v

    def add_port_forwarding(self, service_port, pod_port):
        for f in self.port_forwardings:
            if service_port.name and f.service_port.name == service_port.name:
                log.warning("The port name %s on %s service is already in use. Not adding the new forwarding",
                            service_port.name, self.name)
                return False
            if f.service_port.number == service_port.number:
                log.warning("The port number %d on %s service is already in use. Not adding the new forwarding",
                            service_port.number, self.name)
                return False
        self.port_forwardings.append(PortForwarding(service_port, pod_port))
        return True

    def add_volume(self, volume):
        vols = self.pod_spec.setdefault("volumes", [])
        for v in vols:
            if v.get("name") == volume.get("name"):
                log.debug("Found an existing volume. Ignoring new volume : %r", volume)
                return
        vols.append(volume)

    def has_valid_annotation(self, annotation):
        return bool(self.annotations) and self.annotations.get(annotation) == ANNOTATION_LABEL_VALUE

    def copy(self):
        s = common.shallow_copy(self)
        s.pod_spec = common.deep_copy(self.pod_spec)
        s.annotations = dict(self.annotations) if self.annotations is not None else None
        s.labels = dict(self.labels) if self.labels is not None else None
        s.port_forwardings = [PortForwarding(Port(f.service_port.number, f.service_port.name),
                                             Port(f.pod_port.number, f.pod_port.name)) for f in self.port_forwardings]
        s.networks = list(self.networks)
        return s

    def __repr__(self):
        return "IRService(%s, %r)" % (self.name, self.pod_spec)


def new_service_from_plan_service(ps):
    return Service(ps.service_name, ps.service_rel_path)


def new_service_with_name(name):
    return Service(name, "/" + name)


class Container:
    def __init__(self, container_build_type="", image_name="", new=False):
        self.container_build_type = container_build_type
        self.repo_info = plantypes.RepoInfo()
        self.image_names = [image_name]
        self.new = new
        self.new_files = {}
        self.exposed_ports = []
        self.user_id = -1
        self.accessed_dirs = []

    def merge(self, newc):
        """``Container.Merge`` (ir.go:154-190)."""
        if self.container_build_type != newc.container_build_type:
            return False
        for imagename in newc.image_names:
            if common.is_string_present(self.image_names, imagename):
                if self.new != newc.new:
                    log.error("Both old and new image seems to share the same tag for container %s.", imagename)
                elif self.new and newc.new:
                    for fp, contents in newc.new_files.items():
                        if fp in self.new_files:
                            if self.new_files[fp] != contents:
                                log.error("Two build scripts found for image : %s in %s. Ignoring new script.", imagename, fp)
                        else:
                            self.new_files[fp] = contents
                    if self.user_id != newc.user_id:
                        log.error("Two different users found for image : %d in %d. Ignoring new users.", self.user_id, newc.user_id)
                self.image_names = common.merge_string_slices(self.image_names, newc.image_names)
                self.exposed_ports = common.merge_int_slices(self.exposed_ports, newc.exposed_ports)
                self.accessed_dirs = common.merge_string_slices(self.accessed_dirs, newc.accessed_dirs)
                if not self.new:
                    self.new_files = dict(newc.new_files)
                    self.user_id = newc.user_id
                return True
            log.debug("Mismatching during container merge [%s, %s]", self.image_names, imagename)
        return False

    def add_file(self, path, contents):
        if path in self.new_files:
            if self.new_files[path] != contents:
                log.error("Script already exists for image at %s. Ignoring new script.", path)
        else:
            self.new_files[path] = contents

    def add_exposed_port(self, port):
        if port not in self.exposed_ports:
            self.exposed_ports.append(port)

    def add_image_name(self, name):
        if not common.is_string_present(self.image_names, name):
            self.image_names.append(name)

    def add_accessed_dirs(self, d):
        if not common.is_string_present(self.accessed_dirs, d):
            self.accessed_dirs.append(d)

    def copy(self):
        c = common.shallow_copy(self)
        c.repo_info = self.repo_info.copy()
        c.image_names = list(self.image_names)
        c.new_files = dict(self.new_files)
        c.exposed_ports = list(self.exposed_ports)
        c.accessed_dirs = list(self.accessed_dirs)
        return c

    def __repr__(self):
        return "Container(%s, %r, new=%r, files=%r, ports=%r)" % (
            self.container_build_type, self.image_names, self.new, sorted(self.new_files), self.exposed_ports)


def new_container(container_build_type, image_name, new):
    return Container(container_build_type, image_name, new)


def new_container_from_image_info(info):
    name = info.tags[0] if info.tags else ""
    if not info.tags:
        log.error("The image info %s has no tags. Leaving the tag empty for the container.", info.go_v())
    c = Container(plantypes.REUSE, name, False)
    c.image_names = list(info.tags)
    c.exposed_ports = list(info.ports)
    c.user_id = info.user_id
    c.accessed_dirs = list(info.accessed_dirs)
    return c


class Storage:
    def __init__(self, name="", storage_type="", pvc_spec=None, content=None, annotations=None,
                 secret_type="", string_data=None):
        self.name = name
        self.annotations = annotations
        self.pvc_spec = pvc_spec if pvc_spec is not None else {}
        self.storage_type = storage_type
        self.secret_type = secret_type
        self.content = content
        self.string_data = string_data

    def merge(self, newst):
        if self.name == newst.name:
            if self.content is not None and newst.content is not None:
                self.content = newst.content
            self.storage_type = newst.storage_type
            self.pvc_spec = common.deep_copy(newst.pvc_spec)
            return True
        log.debug("Mismatching storages [%s, %s]", self.name, newst.name)
        return False

    def copy(self):
        s = common.shallow_copy(self)
        s.pvc_spec = common.deep_copy(self.pvc_spec)
        s.content = dict(self.content) if self.content is not None else None
        s.annotations = dict(self.annotations) if self.annotations is not None else None
        s.string_data = dict(self.string_data) if self.string_data is not None else None
        return s

    def __repr__(self):
        return "Storage(%s, %s)" % (self.name, self.storage_type)


class ServiceAccount:
    def __init__(self, name, secret_names=None):
        self.name = name
        self.secret_names = list(secret_names or [])


class RoleBinding:
    def __init__(self, name, role_name, service_account_name):
        self.name = name
        self.role_name = role_name
        self.service_account_name = service_account_name


class PolicyRule:
    def __init__(self, api_groups, resources, verbs):
        self.api_groups = api_groups
        self.resources = resources
        self.verbs = verbs


class Role:
    def __init__(self, name, policy_rules=None):
        self.name = name
        self.policy_rules = list(policy_rules or [])


class TektonResources:
    def __init__(self):
        self.event_listeners = []
        self.trigger_bindings = []
        self.trigger_templates = []
        self.pipelines = []


class IR:
    def __init__(self):
        self.root_dir = ""
        self.name = ""
        self.services = {}
        self.storages = []
        self.containers = []
        self.roles = []
        self.role_bindings = []
        self.service_accounts = []
        self.kubernetes = plantypes.KubernetesOutput()
        self.target_cluster_spec = ClusterMetadataSpec()
        self.cached_objects = []
        self.values = HelmValues()
        self.ingress_tls_secret_name = ""
        self.tekton_resources = TektonResources()
        self.add_copy_sources_warning = False

    def sorted_services(self):
        return [self.services[k] for k in sorted(self.services)]

    def merge(self, new):
        """``IR.Merge`` (ir.go:212-235)."""
        if self.name != new.name and self.name == "":
            self.name = new.name
        self.kubernetes.merge(new.kubernetes)
        for name in sorted(new.services):
            if name in self.services:
                log.warning("Two services of same service name %s. Using the new object.", name)
            self.services[name] = new.services[name]
        for c in new.containers:
            self.add_container(c)
        for s in new.storages:
            self.add_storage(s)
        self.target_cluster_spec.merge(new.target_cluster_spec)
        self.cached_objects.extend(new.cached_objects)
        self.values.merge(new.values)

    def is_ingress_tls_enabled(self):
        return self.ingress_tls_secret_name != ""

    # The reference offers every new container (storage) to each existing one
    # in turn (ir.go:369-380, 387-395), which is quadratic in the number of
    # services.  The first existing container that ``merge`` accepts is the
    # first one of the same build type sharing an image name (case-folded), so
    # an index from (build type, folded name) to list positions finds it
    # directly; storages merge on equal names.  The indexes are rebuilt when
    # the list object is replaced or its length changes behind their back.

    def _container_index(self):
        idx = self.__dict__.get("_cidx")
        if idx is None or idx[0] is not self.containers or idx[1] != len(self.containers):
            buckets = {}
            for pos, c in enumerate(self.containers):
                bt = c.container_build_type
                for n in c.image_names:
                    b = buckets.setdefault((bt, common.go_fold(n)), [])
                    if not b or b[-1] != pos:
                        b.append(pos)
            idx = self._cidx = [self.containers, len(self.containers), buckets]
        return idx

    def add_container(self, container):
        idx = self._container_index()
        buckets = idx[2]
        bt = container.container_build_type
        best = -1
        for n in container.image_names:
            b = buckets.get((bt, common.go_fold(n)))
            if b and (best < 0 or b[0] < best):
                best = b[0]
        if best >= 0:
            c = self.containers[best]
            if c.merge(container):
                for n in c.image_names:
                    b = buckets.setdefault((bt, common.go_fold(n)), [])
                    if best not in b:
                        b.append(best)
                        b.sort()
                return
        pos = len(self.containers)
        self.containers.append(container)
        for n in container.image_names:
            b = buckets.setdefault((bt, common.go_fold(n)), [])
            if not b or b[-1] != pos:
                b.append(pos)
        idx[1] = len(self.containers)

    def add_storage(self, st):
        idx = self.__dict__.get("_sidx")
        if idx is None or idx[0] is not self.storages or idx[1] != len(self.storages):
            first = {}
            for pos, s in enumerate(self.storages):
                first.setdefault(s.name, pos)
            idx = self._sidx = [self.storages, len(self.storages), first]
        pos = idx[2].get(st.name)
        if pos is not None and self.storages[pos].merge(st):
            return
        idx[2].setdefault(st.name, len(self.storages))
        self.storages.append(st)
        idx[1] = len(self.storages)

    def container_finder(self):
        """A :meth:`get_container` over a snapshot of the containers: one pass
        builds a folded-name index, then every lookup is a dict probe.  Valid
        while no container or image name changes (the port-merge optimizer
        asks once per service without touching containers, which made the
        plain scan quadratic in the size of the tree)."""
        first = {}
        first_new = {}
        for pos, c in enumerate(self.containers):
            for n in c.image_names:
                k = common.go_fold(n)
                first.setdefault(k, pos)
                if c.new:
                    first_new.setdefault(k, pos)
        containers = list(self.containers)
        registry = self.kubernetes.registry_url

        def find(imagename):
            best = first.get(common.go_fold(imagename))
            parts = imagename.split("/")
            if len(parts) > 2 and parts[0] == registry:
                p = first_new.get(common.go_fold(parts[-1]))
                if p is not None and (best is None or p < best):
                    best = p
            if best is None:
                return None, False
            return containers[best], True
        return find

    def get_container(self, imagename):
        for c in self.containers:
            if common.is_string_present(c.image_names, imagename):
                return c, True
            if c.new:
                parts = imagename.split("/")
                if len(parts) > 2 and parts[0] == self.kubernetes.registry_url and common.is_string_present(c.image_names, parts[-1]):
                    return c, True
        return None, False

    def copy(self):
        ir = common.shallow_copy(self)
        ir.services = {k: v.copy() for k, v in self.services.items()}
        ir.storages = [s.copy() for s in self.storages]
        ir.containers = [c.copy() for c in self.containers]
        ir.roles = list(self.roles)
        ir.role_bindings = list(self.role_bindings)
        ir.service_accounts = list(self.service_accounts)
        ir.kubernetes = self.kubernetes.copy()
        ir.target_cluster_spec = self.target_cluster_spec.copy()
        ir.cached_objects = common.deep_copy(self.cached_objects)
        ir.values = self.values.copy()
        return ir


def new_ir(plan):
    """``irtypes.NewIR``."""
    ir = IR()
    ir.name = plan.name
    ir.root_dir = plan.root_dir
    ir.kubernetes = plan.kubernetes.copy()
    ir.target_cluster_spec = ClusterMetadataSpec([], {}, "")
    return ir


def empty_ir():
    """``irtypes.IR{Services: map[string]Service{}}`` as built by the compose loaders."""
    ir = IR()
    ir.kubernetes = plantypes.KubernetesOutput()
    ir.kubernetes.artifact_type = ""
    ir.kubernetes.target_cluster_type = ""
    return ir
