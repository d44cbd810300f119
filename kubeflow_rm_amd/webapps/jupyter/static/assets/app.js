// Jupyter web app frontend (reference crud-web-apps/jupyter/frontend): the notebook table (common
// resource table, polled with backoff; "All namespaces" adds a Namespace column), connect / start /
// stop / delete, notebook details (overview + conditions / events / logs viewer / YAML), and the
// spawner built from /api/config: image groups, CPU and memory requests with their limits
// (form-cpu-ram: the admin's limitFactor pre-fills the limit until the user edits it), GPUs (count +
// vendor from the admin's vendor list, /api/gpus marks the vendors installed in the cluster: the
// form-gpus component), workspace volume (name from the {notebook-name} template, size,
// access mode), data volumes (mount follows the volume name until edited), affinity / toleration
// groups, PodDefault configurations, shared memory. Volumes have the "Custom (Advanced)" type of
// form-new/volume/{new,existing}: the PVC (or volume source) is edited as YAML in kf.YamlEditor,
// and the notebook page's YAML tab shows the Notebook or its Pod (pages/notebook-page/yaml).
//
// The `JWA` object holds the pure parts (form defaults, limits, volume naming, request body,
// validation, table columns): node unit-tests them against the reference's Cypress fixtures.
(function (global) {
  "use strict";
  const kf = global.kf || (typeof require !== "undefined" ? require("../../../crud_backend/static/kf.js") : null);
  const ALL = "*all-namespaces*";
  const HOME = "/home/jovyan";

  // ---- pure helpers ---------------------------------------------------------------------------
  const JWA = {
    ALL,
    columns(allNamespaces) {
      const e = kf.esc;
      const cols = [
        { title: "Status", value: (r) => r.status.phase, html: (r) => kf.statusIcon(r.status) },
        { title: "Name", value: (r) => r.name, html: (r) => kf.nameLink(r) },
      ];
      if (allNamespaces) cols.push({ title: "Namespace", value: (r) => r.namespace });
      // index-default/config.ts: Created at / Last activity are DateTimeValues, Memory a MemoryValue
      cols.push(
        { title: "Type", value: (r) => r.serverType },
        { title: "Created at", kind: "date", value: (r) => r.age },
        { title: "Last activity", kind: "date", value: (r) => r.last_activity },
        { title: "Image", value: (r) => r.shortImage, html: (r) => `<span title="${e(r.image)}">${e(r.shortImage)}</span>` },
        { title: "GPUs", value: (r) => (r.gpus || {}).count || 0, html: (r) => `<span title="${e((r.gpus || {}).message || "")}">${e((r.gpus || {}).count || 0)}</span>` },
        { title: "CPUs", value: (r) => r.cpu },
        { title: "Memory", kind: "memory", value: (r) => r.memory },
      );
      return cols;
    },
    // confirm dialogs (services/config.ts)
    dialogs: {
      delete: (name) => ({ title: `Are you sure you want to delete this notebook server? ${name}`,
                           message: "Warning: Your data might be lost if the notebook server is not backed by persistent storage",
                           accept: "DELETE", confirmColor: "warn", cancel: "CANCEL", error: "", applying: "DELETING", width: "600px" }),
      stop: (name) => ({ title: `Are you sure you want to stop this notebook server? ${name}`,
                         message: "Warning: Your data might be lost if the notebook server is not backed by persistent storage.",
                         accept: "STOP", confirmColor: "primary", cancel: "CANCEL", error: "", applying: "STOPPING", width: "600px" }),
    },
    // "{notebook-name}-workspace" -> "<name>-workspace" ("-workspace" while the name is empty)
    volumeName(template, notebookName) { return String(template || "").split("{notebook-name}").join(notebookName || ""); },
    // "20Gi" -> {size: "20", unit: "Gi"}
    splitSize(q) {
      const m = String(q || "").match(/^([0-9.]+)\s*([A-Za-z]*)$/);
      return m ? { size: m[1], unit: m[2] || "Gi" } : { size: "", unit: "Gi" };
    },
    mountFor(volumeName) { return `${HOME}/${volumeName}`; },
    // limit = request x factor, one decimal (form.py _limit); "" when the admin set no factor
    limitFrom(request, factor, unit) {
      if (!factor || factor === "none" || request === "" || request == null) return "";
      const v = parseFloat(String(request).replace(unit || "", ""));
      if (isNaN(v)) return "";
      return `${Math.round(v * parseFloat(factor) * 10) / 10}${unit || ""}`;
    },
    formDefaults(config, notebookName) {
      const c = config || {};
      const ws = ((c.workspaceVolume || {}).value) || {};
      const pvc = ws.newPvc || {};
      const size = JWA.splitSize((((pvc.spec || {}).resources || {}).requests || {}).storage);
      const gpu = ((c.gpus || {}).value) || {};
      const cpu = String(((c.cpu || {}).value) || "0.5"), mem = String(((c.memory || {}).value) || "1.0Gi");
      return {
        name: notebookName || "", serverType: "jupyter",
        image: ((c.image || {}).value) || "", imageGroupOne: ((c.imageGroupOne || {}).value) || "",
        imageGroupTwo: ((c.imageGroupTwo || {}).value) || "", customImage: "",
        imagePullPolicy: ((c.imagePullPolicy || {}).value) || "IfNotPresent",
        cpu, cpuLimit: JWA.limitFrom(cpu, (c.cpu || {}).limitFactor, ""),
        memory: mem, memoryLimit: JWA.limitFrom(mem, (c.memory || {}).limitFactor, "Gi"),
        gpus: { num: gpu.num || "none", vendor: gpu.vendor || "" },  // form-new: config.gpus.value.vendor as is
        shm: !!((c.shm || {}).value),
        workspace: ws.newPvc || ws.existingSource ? {
          enabled: true, type: ws.existingSource ? "existing" : "new", template: (pvc.metadata || {}).name || "{notebook-name}-workspace",
          name: JWA.volumeName((pvc.metadata || {}).name || "{notebook-name}-workspace", notebookName),
          size: size.size, unit: size.unit, accessMode: ((pvc.spec || {}).accessModes || ["ReadWriteOnce"])[0],
          // volume/new/storage-class: "Use default class" unless the admin's PVC names a class
          useDefaultSC: !("storageClassName" in (pvc.spec || {})), storageClass: (pvc.spec || {}).storageClassName || "",
          mount: ws.mount || HOME, existing: ((ws.existingSource || {}).persistentVolumeClaim || {}).claimName || "",
        } : { enabled: false },
        datavols: [],
        affinityConfig: ((c.affinityConfig || {}).value) || "none",
        tolerationGroup: ((c.tolerationGroup || {}).value) || "none",
        configurations: (((c.configurations || {}).value) || []).slice(),
      };
    },
    // a new data volume row; its mount tracks the name until the user types in the mount field
    newDataVolume(notebookName, index) {
      const name = `${notebookName || ""}-datavol-${index}`;
      return { type: "new", name, size: "5", unit: "Gi", accessMode: "ReadWriteOnce", mount: JWA.mountFor(name), mountDirty: false, existing: "",
               useDefaultSC: true, storageClass: "" };
    },
    renameDataVolume(vol, name) {
      const out = Object.assign({}, vol, { name });
      if (!vol.mountDirty) out.mount = JWA.mountFor(name);
      return out;
    },
    editMount(vol, mount) { return Object.assign({}, vol, { mount, mountDirty: true }); },
    // the newPvc / existingSource a volume row describes (what "Custom (Advanced)" starts from)
    volumeSpec(v) {
      if (v.type === "existing") return { persistentVolumeClaim: { claimName: v.existing } };
      const spec = { resources: { requests: { storage: `${v.size}${v.unit}` } }, accessModes: [v.accessMode] };
      // a disabled storage-class control (use the default) leaves the field out of the PVC
      if (v.useDefaultSC === false) spec.storageClassName = v.storageClass || "";
      return { metadata: { name: v.template || v.name }, spec };
    },
    // the class select: "Empty storage class" (value "") and the cluster's classes; while "Use
    // default class" is ticked it is disabled and shows the default
    storageClassOptions(classes, v, defaultClass) {
      const cur = v.useDefaultSC === false ? (v.storageClass || "") : (defaultClass || "");
      return [`<option value=""${cur === "" ? " selected" : ""}>Empty storage class</option>`]
        .concat((classes || []).map((c) => `<option value="${kf.esc(c)}"${c === cur ? " selected" : ""}>${kf.esc(c)}</option>`)).join("");
    },
    // typeChanged(CUSTOM): dump the current spec into the editor; back to the plain form drops it
    toCustom(v) { const spec = JWA.volumeSpec(v); return Object.assign({}, v, { custom: true, yaml: kf.toYaml(spec), spec, yamlError: "" }); },
    fromCustom(v) { return Object.assign({}, v, { custom: false, yaml: "", spec: undefined, yamlError: "" }); },
    // set yaml(text): a parse error is shown and keeps the last good spec (the form also refuses
    // to submit while it is shown, where the reference would send the stale spec)
    editCustom(v, text) {
      const [parsed, error] = kf.parseYaml(text);
      return Object.assign({}, v, { yaml: text, yamlError: error, spec: error ? v.spec : parsed });
    },
    kindOptions(v) {
      const opts = v.type === "existing" ? [["pvc", "Kubernetes Volume"], ["custom", "Custom (Advanced)"]]
        : [["empty", "Empty volume"], ["custom", "Custom (Advanced)"]];
      return opts.map(([val, label]) => `<option value="${val}"${(val === "custom") === !!v.custom ? " selected" : ""}>${label}</option>`).join("");
    },
    // notebook-page/yaml: the Notebook or its Pod, with the component's placeholder texts
    yamlTabText(selection, notebook, pod, podRequestCompleted) {
      if (selection === "pod") {
        if (pod) return kf.toYaml(pod);
        return podRequestCompleted ? "No pod available for this notebook." : "Pod information is still being loaded.";
      }
      return notebook ? kf.toYaml(notebook) : "No data has been found...";
    },
    // form-gpus.component.ts: the admin's vendor list; a vendor /api/gpus does not report as
    // installed keeps its option but carries the "no GPUs" tooltip; the vendor control is disabled
    // while the count is "none", and a count needs a vendor (vendorWithNum -> vendorNullName)
    gpuVendors(config) { return ((((config || {}).gpus || {}).value || {}).vendors) || []; },
    vendorTooltip(vendor, installed) {
      return installed && installed.has && installed.has(vendor.limitsKey) ? ""
        : `There are currently no ${vendor.uiName} GPUs in your cluster.`;
    },
    vendorDisabled(gpus) { return !gpus || gpus.num === "none"; },
    vendorError(gpus) {
      return gpus && gpus.num !== "none" && !gpus.vendor ? "You must also specify the GPU Vendor for the assigned GPUs" : "";
    },
    vendorOptions(config, gpus, installed) {
      const e = kf.esc;
      const vendors = JWA.gpuVendors(config);
      const empty = !gpus.vendor || !vendors.some((v) => v.limitsKey === gpus.vendor) ? '<option value=""></option>' : "";
      return empty + vendors.map((v) => `<option value="${e(v.limitsKey)}" title="${e(JWA.vendorTooltip(v, installed))}"` +
        `${v.limitsKey === gpus.vendor ? " selected" : ""}>${e(v.uiName)}</option>`).join("");
    },
    validate(f) {
      const errs = [];
      const n = kf.validators.name(f.name, 52);  // StatefulSet pod names: <name>-0 within 63
      if (n) errs.push(n);
      for (const [what, v, lim, check] of [["CPU", f.cpu, f.cpuLimit, kf.validators.cpu], ["Memory", f.memory, f.memoryLimit, kf.validators.memory]]) {
        const e1 = check(v);
        if (e1) errs.push(e1);
        if (lim) {
          const e2 = check(lim) || kf.validators.limitAtLeastRequest(v, lim, what);
          if (e2) errs.push(e2);
        }
      }
      const ve = JWA.vendorError(f.gpus);
      if (ve) errs.push(ve);
      if (f.workspace && f.workspace.enabled && f.workspace.custom && f.workspace.yamlError) errs.push(`Workspace volume: ${f.workspace.yamlError}`);
      (f.datavols || []).forEach((d) => {
        if (d.custom && d.yamlError) errs.push(`Data volume: ${d.yamlError}`);
        if (d.type === "new" && !d.custom && kf.validators.name(d.name)) errs.push(`Data volume: ${kf.validators.name(d.name)}`);
        if (!String(d.mount || "").startsWith("/")) errs.push(`Data volume mount must be an absolute path: ${d.mount}`);
      });
      return errs;
    },
    // POST /api/namespaces/<ns>/notebooks body (backend form.py contract)
    buildBody(f, config, namespace) {
      const image = f.serverType === "group-one" ? f.imageGroupOne : f.serverType === "group-two" ? f.imageGroupTwo : f.image;
      const vol = (v) => (v.custom ? (v.type === "existing" ? { mount: v.mount, existingSource: v.spec } : { mount: v.mount, newPvc: v.spec })
        : v.type === "existing" ? { mount: v.mount, existingSource: JWA.volumeSpec(v) } : { mount: v.mount, newPvc: JWA.volumeSpec(v) });
      const body = {
        name: f.name, namespace, serverType: f.serverType,
        image: f.customImage ? f.customImage.trim() : image, customImage: !!f.customImage,
        imagePullPolicy: f.imagePullPolicy, cpu: String(f.cpu), memory: String(f.memory),
        gpus: f.gpus.num === "none" ? { num: "none" } : { num: String(f.gpus.num), vendor: f.gpus.vendor },
        tolerationGroup: f.tolerationGroup || "none", affinityConfig: f.affinityConfig || "none",
        shm: !!f.shm, configurations: (f.configurations || []).slice(), datavols: (f.datavols || []).map(vol),
      };
      if (f.cpuLimit) body.cpuLimit = String(f.cpuLimit);
      if (f.memoryLimit) body.memoryLimit = String(f.memoryLimit);
      if (f.workspace && f.workspace.enabled) body.workspace = vol(f.workspace);
      // fields the admin pinned readOnly must not be sent (form.py get_form_value -> 400)
      const ro = { cpu: "cpu", memory: "memory", gpus: "gpus", shm: "shm", imagePullPolicy: "imagePullPolicy",
                   tolerationGroup: "tolerationGroup", affinityConfig: "affinityConfig", configurations: "configurations",
                   workspace: "workspaceVolume", datavols: "dataVolumes" };
      Object.keys(ro).forEach((k) => { if (((config || {})[ro[k]] || {}).readOnly) delete body[k]; });
      if (((config || {}).cpu || {}).readOnly) delete body.cpuLimit;
      if (((config || {}).memory || {}).readOnly) delete body.memoryLimit;
      return body;
    },
    // ---- notebook page overview (notebook-page/overview): the main container's requests and
    // limits, type, creator, shared memory, volumes grouped by kind, the PodDefault
    // "configurations" the notebook's labels select, and the env grouped by where it came from
    mainContainer(nb) {
      const cs = ((((nb || {}).spec || {}).template || {}).spec || {}).containers || [];
      return cs.find((c) => c.name === ((nb || {}).metadata || {}).name) || null;
    },
    overview(nb) {
      const ann = ((nb || {}).metadata || {}).annotations || {};
      const c = JWA.mainContainer(nb);
      const res = (c || {}).resources || {};
      const vols = ((((nb || {}).spec || {}).template || {}).spec || {}).volumes;
      const type = ann["notebooks.kubeflow.org/server-type"];
      return {
        notebookType: !type ? "empty" : ({ "group-two": "RStudio", "group-one": "VSCode", jupyter: "JupyterLab" }[type] || type),
        sharedMemory: !vols ? "null" : vols.some((v) => v.name === "dshm") ? "Yes" : "No",
        notebookCreator: ann["notebooks.kubeflow.org/creator"] || null,
        cpuRequests: (res.requests || {}).cpu || null, cpuLimits: (res.limits || {}).cpu || null,
        memoryRequests: (res.requests || {}).memory || null, memoryLimits: (res.limits || {}).memory || null,
        dockerImage: (c || {}).image || null,
      };
    },
    VOLUME_GROUPS: {
      PersistentVolumeClaims: ["Storage claimed from a PersistentVolume: it outlives the pod, with a requested size and access mode.",
        "https://kubernetes.io/docs/concepts/storage/persistent-volumes/"],
      "Memory-backed Volumes": ["An emptyDir on tmpfs: fast, counted against the container's memory limit, gone with the pod.",
        "https://kubernetes.io/docs/concepts/storage/volumes/#emptydir"],
      Ephemerals: ["An emptyDir: scratch space created empty with the pod on its node and deleted with it.",
        "https://kubernetes.io/docs/concepts/storage/volumes/#emptydir"],
      ConfigMaps: ["Configuration data from a ConfigMap, mounted as files.", "https://kubernetes.io/docs/concepts/storage/volumes/#configmap"],
      Secrets: ["Sensitive data from a Secret, mounted as files on tmpfs.", "https://kubernetes.io/docs/concepts/storage/volumes/#secret"],
      "Other Volumes": ["", "https://kubernetes.io/docs/concepts/storage/volumes"],
    },
    classifyVolume(v) {
      if (v.persistentVolumeClaim) return "PersistentVolumeClaims";
      if (v.emptyDir && v.emptyDir.medium === "Memory") return "Memory-backed Volumes";
      if (v.emptyDir) return "Ephemerals";
      if (v.configMap) return "ConfigMaps";
      if (v.secret) return "Secrets";
      return "Other Volumes";
    },
    // [{name, info, url, items: [{name, url?}]}], PVCs first (links to the volumes app's details)
    volGroups(nb) {
      const groups = [];
      const ns = ((nb || {}).metadata || {}).namespace;
      (((((nb || {}).spec || {}).template || {}).spec || {}).volumes || []).forEach((v) => {
        const name = JWA.classifyVolume(v);
        const item = name === "PersistentVolumeClaims" ? { name: v.name, url: `/volumes/volume/details/${ns}/${v.name}` } : { name: v.name };
        let g = groups.find((x) => x.name === name);
        if (!g) {
          const [info, url] = JWA.VOLUME_GROUPS[name];
          g = { name, info, url, items: [] };
          if (name === "PersistentVolumeClaims") groups.unshift(g); else groups.push(g);
        }
        g.items.push(item);
      });
      return groups;
    },
    // PodDefaults whose (first) selector label the notebook carries
    configurations(nb, podDefaults) {
      const labels = Object.keys(((nb || {}).metadata || {}).labels || {});
      return (podDefaults || []).filter((pd) => labels.includes(Object.keys((((pd.spec || {}).selector || {}).matchLabels) || {})[0]))
        .map((pd) => ({ name: pd.metadata.name, Description: pd.spec.desc, Selector: pd.spec.selector, Env: pd.spec.env,
                        Volumes: pd.spec.volumes, VolumeMounts: pd.spec.volumeMounts, ServiceAccountName: pd.spec.serviceAccountName }));
    },
    podDefaultsMessage(podRequestCompleted, configurations) {
      return podRequestCompleted === true && !(configurations || []).length ? "No configurations available for this notebook." : "";
    },
    // configuration-info-dialog: the configuration minus its name, as YAML
    configurationYaml(config) {
      if (!config) return "No information available about the configuration";
      const c = Object.assign({}, config);
      delete c.name;
      Object.keys(c).forEach((k) => { if (c[k] === undefined) delete c[k]; });
      return kf.toYaml(c);
    },
    // env chips: "Notebook CR" (the CR's own env), then per PodDefault "(Configuration)" and "Other"
    // for what the pod has beyond the CR; valueFrom.fieldRef resolves against the pod
    envGroups(nb, pod, podDefaults) {
      const chip = (e, obj) => {
        if (e.value) return `${e.name}: ${e.value}`;
        if (e.valueFrom && e.valueFrom.fieldRef) {
          const v = e.valueFrom.fieldRef.fieldPath.split(".").reduce((o, k) => (o == null ? undefined : o[k]), obj);
          return `${e.name}: ${v}`;
        }
        return `${e.name}: undefined`;
      };
      const groups = [];
      const c = JWA.mainContainer(nb);
      const crChips = c && c.env ? c.env.map((e) => chip(e, pod)) : [];
      if (c && c.env) groups.push({ name: "Notebook CR", chips: crChips });
      if (pod && podDefaults) {
        const pc = ((pod.spec || {}).containers || []).find((x) => x.name === ((pod.metadata || {}).labels || {})["notebook-name"]);
        if (pc && pc.env) {
          const pdGroups = podDefaults.map((pd) => ({ name: `${pd.metadata.name} (Configuration)`, pd, chips: [] }));
          const other = { name: "Other", chips: [] };
          pc.env.forEach((e) => {
            const v = chip(e, pod);
            if (crChips.includes(v)) return;
            const g = pdGroups.find((x) => (((x.pd.spec || {}).env) || []).some((pe) => pe.name === e.name)) || other;
            if (!g.chips.includes(v)) g.chips.push(v);
          });
          pdGroups.concat([other]).forEach((g) => { if (g.chips.length) groups.push({ name: g.name, chips: g.chips }); });
        }
      }
      return groups;
    },
    // the union of several namespaces' notebook lists (all-namespaces view)
    merge(lists) { return [].concat(...lists); },
    // index-default.component.ts updateNotebookFields: button states derived from the phase
    // (start/stop "uninitialized" = the Stop form of the toggle, "ready" = Start).
    actionStates(r) {
      const p = r.status.phase;
      return {
        deleteAction: p === "terminating" ? "terminating" : "ready",
        connectAction: p === "ready" ? "ready" : "unavailable",
        startStopAction: p === "ready" ? "uninitialized" : p === "stopped" ? "ready" : p === "terminating" ? "unavailable" : "uninitialized",
      };
    },
    // Optimistic row after an accepted action, until the next poll (startNotebook/stopNotebook/delete).
    markPending(r, what) {
      const next = { delete: ["terminating", "Preparing to delete the Notebook."],
                     start: ["waiting", "Starting the Notebook Server."],
                     stop: ["waiting", "Preparing to stop the Notebook Server."] }[what];
      r.status = Object.assign({}, r.status, { phase: next[0], message: next[1] });
      return Object.assign(r, JWA.actionStates(r));
    },
  };

  // ---- DOM ------------------------------------------------------------------------------------
  function app() {
    const $ = (id) => document.getElementById(id);
    let config = null, poller = null, table = null, namespaces = [], form = null, rows = [];
    let installedVendors = new Set();

    async function loadNamespaces() {
      try { namespaces = (await kf.call("GET", "/api/namespaces")).namespaces; }
      catch (e) { namespaces = kf.namespace() ? [kf.namespace()] : []; }  // not cluster-wide: the dashboard drives it
      const sel = $("ns");
      sel.innerHTML = namespaces.map((n) => `<option value="${kf.esc(n)}">${kf.esc(n)}</option>`).join("") +
        (namespaces.length > 1 ? `<option value="${ALL}">All namespaces</option>` : "");
      if (!kf.namespace() && namespaces.length) kf.setNamespace(namespaces[0]);
      sel.value = kf.namespace();
      sel.onchange = () => { if (sel.value === ALL) { setAll(true); } else { setAll(false); kf.setNamespace(sel.value); } };
    }
    let allNs = false;
    function setAll(v) {
      allNs = v;
      table = new kf.ResourceTable($("notebooks"), tableConfig());
      poller.reset();
    }
    function tableConfig() {
      return {
        columns: JWA.columns(allNs), empty: "No notebooks in this namespace.",
        actions: [
          { name: "connect", label: "Connect", enabled: (r) => r.connectAction === "ready" },
          { name: "toggle", label: (r) => (r.status.phase === "stopped" ? "Start" : "Stop"), enabled: (r) => r.startStopAction !== "unavailable" },
          { name: "delete", label: "Delete", enabled: (r) => r.deleteAction === "ready" },
        ],
        onOpen: (r) => (r.status.phase === "terminating"
          ? kf.snack("Notebook is being deleted, cannot show details.", "INFO") : showDetails(r.namespace, r.name)),
        onAction: (name, r) => {
          if (name === "connect") window.open(`/notebook/${r.namespace}/${r.name}/`);
          const url = `/api/namespaces/${r.namespace}/notebooks/${r.name}`;
          // starting needs no confirmation; stopping and deleting go through the confirm dialog,
          // which stays open with the backend's error if the call fails
          const pending = (what) => (resp) => { if (resp === "accept") { JWA.markPending(r, what); table.setRows(rows); } poller.reset(); };
          if (name === "toggle" && r.status.phase === "stopped") {
            JWA.markPending(r, "start"); table.setRows(rows);
            act("PATCH", r.namespace, r.name, { stopped: false });
          } else if (name === "toggle") kf.confirmDialog(JWA.dialogs.stop(r.name), () => kf.call("PATCH", url, { stopped: true })).then(pending("stop"));
          if (name === "delete") kf.confirmDialog(JWA.dialogs.delete(r.name), () => kf.call("DELETE", url)).then(pending("delete"));
        },
      };
    }

    async function refresh() {
      const list = allNs ? namespaces : [kf.namespace()].filter(Boolean);
      if (!list.length) return null;
      rows = JWA.merge(await Promise.all(list.map(async (ns) =>
        (await kf.call("GET", `/api/namespaces/${ns}/notebooks`)).notebooks.map((r) => Object.assign({ namespace: ns }, r)))))
        .map((r) => Object.assign(r, JWA.actionStates(r)));
      table.setRows(rows);
      return rows.map((r) => [r.namespace, r.name, r.status.phase]);
    }

    // notebook page: overview + conditions / events / logs / YAML (JWA pages/notebook-page)
    function showDetails(ns, name) {
      const base = `/api/namespaces/${ns}/notebooks/${name}`;
      const e = kf.esc;
      let logs = null;
      return kf.details(`Notebook ${ns}/${name}`, [
        { name: "Overview", render: async () => {
          if (logs) logs.stop();
          const nb = (await kf.call("GET", base)).notebook;
          let pod = null, podDone = false, pds = null;
          try { pod = (await kf.call("GET", `${base}/pod`)).pod; } catch (err) { /* no pod (stopped or starting) */ }
          podDone = true;
          try { pds = (await kf.call("GET", `/api/namespaces/${ns}/poddefaults`)).poddefaults; } catch (err) { pds = []; }
          const ov = JWA.overview(nb);
          const spec = ((nb.spec || {}).template || {}).spec || {};
          const lim = ((JWA.mainContainer(nb) || {}).resources || {}).limits || {};
          const ann = (nb.metadata || {}).annotations || {};
          const st = nb.status || {};
          const configs = JWA.configurations(nb, pds);
          setTimeout(() => {
            document.querySelectorAll("#kf-details .tab-body button.config-link").forEach((b) => {
              b.onclick = () => {  // configuration-info-dialog
                const cfg = configs[Number(b.dataset.i)];
                kf.infoDialog(`${cfg.name}: `, cfg.Description, kf.yamlHtml(JWA.configurationYaml(cfg), 280), "600px");
              };
            });
          }, 0);
          const rows = [["Name", nb.metadata.name], ["Namespace", nb.metadata.namespace], ["Created", nb.metadata.creationTimestamp],
            ["Type", ov.notebookType], ["Shared memory enabled", ov.sharedMemory]];
          if (ov.notebookCreator) rows.push(["Notebook creator", ov.notebookCreator]);
          for (const [k, v] of [["Minimum CPU", ov.cpuRequests], ["Maximum CPU", ov.cpuLimits], ["Minimum memory", ov.memoryRequests], ["Maximum memory", ov.memoryLimits]])
            if (v) rows.push([k, v]);
          rows.push(["Image", ov.dockerImage], ["MI355X GPUs", lim["amd.com/gpu"] || "0"], ["Allocated GPU ids", st.gpus || "-"],
            ["Ready replicas", st.readyReplicas || 0], ["Last activity", ann["notebooks.kubeflow.org/last-activity"] || "-"],
            ["Cold start (ms)", ann["notebooks.kubeflow.org/cold-start-phases"] || "-"], ["Stopped", ann["kubeflow-resource-stopped"] || "no"]);
          const groups = JWA.volGroups(nb);
          const volHtml = groups.length ? groups.map((g) => `<div class="vol-group"><b title="${e(g.info + (g.info ? " " : "") + "Read more at " + g.url)}">${e(g.name)}</b> ` +
            g.items.map((i) => (i.url ? `<a class="vol-link" href="${e(i.url)}">${e(i.name)}</a>` : `<span class="chip">${e(i.name)}</span>`)).join(" ") + "</div>").join("")
            : '<p class="muted">No volumes available for this notebook.</p>';
          const cfgHtml = configs.map((c, i) => `<button type="button" class="config-link lib-link" data-i="${i}">${e(c.name)}</button>`).join(" ") +
            `<span class="muted">${e(JWA.podDefaultsMessage(podDone, configs))}</span>`;
          const env = JWA.envGroups(nb, pod, pds);
          const envHtml = env.length ? env.map((g) => `<div class="env-group"><b>${e(g.name)}</b> ${g.chips.map((c) => `<span class="chip">${e(c)}</span>`).join(" ")}</div>`).join("")
            : '<p class="muted">No environment variables available for this notebook.</p>';
          return kf.kvTable(rows) + `<h3>Volumes</h3>${volHtml}<h3>Configurations</h3><div class="configurations">${cfgHtml}</div>` +
            `<h3>Environment</h3>${envHtml}` +
            (st.gpuReadiness ? `<h3>GPU readiness op</h3>${kf.yamlHtml(kf.toYaml(st.gpuReadiness), 200)}` : "") +
            `<h3>Conditions</h3>${kf.conditionsTable(st.conditions)}`;
        } },
        { name: "Events", render: async () => { if (logs) logs.stop(); return kf.eventsTable((await kf.call("GET", `${base}/events`)).events); } },
        { name: "Logs", render: async () => {
          const pod = (await kf.call("GET", `${base}/pod`)).pod;
          setTimeout(() => {
            const el = document.querySelector("#kf-details .tab-body .logs-host");
            if (!el) return;
            logs = new kf.LogsViewer(el, async () => (await kf.call("GET", `${base}/pod/${pod.metadata.name}/logs`)).logs).follow();
          }, 0);
          return `<p class="muted">Pod ${e(pod.metadata.name)} (following)</p><div class="logs-host"></div>`;
        } },
        { name: "YAML", render: async () => {
          if (logs) logs.stop();
          const nb = (await kf.call("GET", base)).notebook;
          let pod = null, podDone = false;
          const podReq = kf.call("GET", `${base}/pod`).then((r) => { pod = r.pod; }, () => {}).then(() => { podDone = true; });
          setTimeout(() => {
            const host = document.querySelector("#kf-details .tab-body .yaml-host");
            const sel = document.querySelector("#kf-details .tab-body select.yaml-which");
            if (!host || !sel) return;
            const ed = new kf.YamlEditor(host, { readOnly: true, height: 490, text: JWA.yamlTabText("notebook", nb) });
            const show = () => ed.setText(JWA.yamlTabText(sel.value, nb, pod, podDone));
            sel.onchange = show;
            podReq.then(() => { if (sel.value === "pod") show(); });
          }, 0);
          return '<div class="yaml-tab"><p class="message">Show the full YAML of the <select class="yaml-which">' +
            '<option value="notebook">Notebook</option><option value="pod">Pod</option></select></p><div class="yaml-host"></div></div>';
        } },
      ]);
    }

    async function act(method, ns, name, body) {
      try { await kf.call(method, `/api/namespaces/${ns}/notebooks/${name}`, body); }
      catch (e) { kf.snack(e.message, "ERROR"); }
      poller.reset();
    }

    // ---- spawner ----
    function renderDataVolumes() {
      const host = $("f-datavols");
      const hide = (d, when) => (when || d.custom ? " hidden" : "");
      host.innerHTML = form.datavols.map((d, i) => `<div class="datavol${i === form.datavols.length - 1 ? " last" : ""}" data-cy="data volumes" data-i="${i}">
        <select class="dv-type"><option value="new"${d.type === "new" ? " selected" : ""}>new</option><option value="existing"${d.type === "existing" ? " selected" : ""}>existing</option></select>
        <select class="dv-kind" title="Custom (Advanced): edit the K8s ${d.type === "existing" ? "volume" : "PVC full"} spec">${JWA.kindOptions(d)}</select>
        <input class="dv-name" data-cy="volume name input" value="${kf.esc(d.name)}" size="16"${hide(d, d.type === "existing")}>
        <select class="dv-existing"${hide(d, d.type !== "existing")}>${(form.pvcs || []).map((p) => `<option${p.name === d.existing ? " selected" : ""}>${kf.esc(p.name)}</option>`).join("")}</select>
        <input class="dv-size" value="${kf.esc(d.size)}" size="4"${hide(d, d.type === "existing")}><span class="muted"${hide(d, d.type === "existing")}>Gi</span>
        <select class="dv-mode"${hide(d, d.type === "existing")}>${["ReadWriteOnce", "ReadWriteMany", "ReadOnlyMany"].map((m) => `<option${m === d.accessMode ? " selected" : ""}>${m}</option>`).join("")}</select>
        <label class="muted"${hide(d, d.type === "existing")}><input type="checkbox" class="dv-sc-default"${d.useDefaultSC !== false ? " checked" : ""}> Use default class</label>
        <select class="dv-sc" title="Storage class"${hide(d, d.type === "existing")}${d.useDefaultSC !== false ? " disabled" : ""}>${JWA.storageClassOptions(form.storageClasses, d, form.defaultStorageClass)}</select>
        <input class="dv-mount" data-cy="mount path" value="${kf.esc(d.mount)}" size="20"><button type="button" class="dv-rm">&times;</button>
        ${d.custom ? `<div class="dv-custom"><p class="muted">Check the K8s docs for the supported volumes and their specs</p><div class="dv-yaml"></div></div>` : ""}</div>`).join("");
      host.querySelectorAll(".datavol").forEach((row) => {
        const i = Number(row.dataset.i);
        const yhost = row.querySelector(".dv-yaml");
        if (yhost) new kf.YamlEditor(yhost, { text: form.datavols[i].yaml, height: 250, onChange: (t) => { form.datavols[i] = JWA.editCustom(form.datavols[i], t); } });
        row.querySelector(".dv-kind").onchange = (ev) => {
          form.datavols[i] = ev.target.value === "custom" ? JWA.toCustom(form.datavols[i]) : JWA.fromCustom(form.datavols[i]);
          renderDataVolumes();
        };
        row.querySelector(".dv-type").onchange = (ev) => { form.datavols[i] = JWA.fromCustom(Object.assign(form.datavols[i], { type: ev.target.value })); if (ev.target.value === "existing" && form.pvcs && form.pvcs[0]) form.datavols[i].existing = form.pvcs[0].name; renderDataVolumes(); };
        row.querySelector(".dv-name").oninput = (ev) => { form.datavols[i] = JWA.renameDataVolume(form.datavols[i], ev.target.value); row.querySelector(".dv-mount").value = form.datavols[i].mount; };
        row.querySelector(".dv-existing").onchange = (ev) => { form.datavols[i].existing = ev.target.value; };
        row.querySelector(".dv-size").oninput = (ev) => { form.datavols[i].size = ev.target.value; };
        row.querySelector(".dv-mode").onchange = (ev) => { form.datavols[i].accessMode = ev.target.value; };
        row.querySelector(".dv-sc-default").onchange = (ev) => { form.datavols[i].useDefaultSC = ev.target.checked; renderDataVolumes(); };
        row.querySelector(".dv-sc").onchange = (ev) => { form.datavols[i].storageClass = ev.target.value; };
        row.querySelector(".dv-mount").oninput = (ev) => { form.datavols[i] = JWA.editMount(form.datavols[i], ev.target.value); };
        row.querySelector(".dv-rm").onclick = () => { form.datavols.splice(i, 1); renderDataVolumes(); };
      });
    }
    function renderWorkspace() {
      const w = form.workspace;
      $("f-ws").checked = !!w.enabled;
      $("f-ws-panel").hidden = !w.enabled;
      $("f-ws-header").textContent = w.enabled ? (w.custom ? "custom" : w.type === "existing" ? w.existing : w.name) : "none";
      $("f-ws-kind").innerHTML = JWA.kindOptions(w);
      $("f-ws-fields").hidden = !!w.custom;
      $("f-ws-custom").hidden = !w.custom;
      if (w.custom) new kf.YamlEditor($("f-ws-yaml"), { text: w.yaml, height: 250, onChange: (t) => { form.workspace = JWA.editCustom(form.workspace, t); } });
      $("f-ws-name").value = w.name || "";
      $("f-ws-size").value = w.size || "";
      $("f-ws-sc-default").checked = w.useDefaultSC !== false;
      $("f-ws-sc").innerHTML = JWA.storageClassOptions(form.storageClasses, w, form.defaultStorageClass);
      $("f-ws-sc").disabled = w.useDefaultSC !== false;
      document.querySelectorAll('input[name="f-ws-mode"]').forEach((r) => { r.checked = r.value === w.accessMode; });
    }
    function fillSpawner() {
      const opts = (list, value) => (list || []).map((i) => `<option${i === value ? " selected" : ""}>${kf.esc(i)}</option>`).join("");
      $("f-image").innerHTML = opts(config.image.options, config.image.value);
      $("f-image-g1").innerHTML = opts((config.imageGroupOne || {}).options, (config.imageGroupOne || {}).value);
      $("f-image-g2").innerHTML = opts((config.imageGroupTwo || {}).options, (config.imageGroupTwo || {}).value);
      $("f-custom-row").hidden = config.allowCustomImage === false;
      const counts = (config.gpus.value || {}).options || ["none", "1", "2", "4", "8"];
      $("f-gpus").innerHTML = counts.map((c) => `<option${c === form.gpus.num ? " selected" : ""}>${c}</option>`).join("");
      renderVendor();
      $("f-cpu").value = form.cpu; $("f-cpu-limit").value = form.cpuLimit;
      $("f-mem").value = form.memory; $("f-mem-limit").value = form.memoryLimit;
      $("f-shm").checked = form.shm;
      const groups = (key) => ['<option value="none">None</option>'].concat(((config[key] || {}).options || [])
        .map((o) => `<option value="${kf.esc(o.configKey)}"${o.configKey === (config[key] || {}).value ? " selected" : ""}>${kf.esc(o.displayName || o.configKey)}</option>`)).join("");
      $("f-affinity").innerHTML = groups("affinityConfig");
      $("f-toleration").innerHTML = groups("tolerationGroup");
      for (const [id, key] of [["f-cpu", "cpu"], ["f-cpu-limit", "cpu"], ["f-mem", "memory"], ["f-mem-limit", "memory"], ["f-gpus", "gpus"], ["f-shm", "shm"]])
        $(id).disabled = !!(config[key] || {}).readOnly;
      renderWorkspace();
      renderDataVolumes();
    }
    function renderVendor() {
      $("f-gpu-vendor").innerHTML = JWA.vendorOptions(config, form.gpus, installedVendors);
      $("f-gpu-vendor").disabled = JWA.vendorDisabled(form.gpus) || !!(config.gpus || {}).readOnly;
      $("f-gpu-vendor-err").textContent = "";
    }
    let cpuLimitDirty = false, memLimitDirty = false;
    function bindSpawner() {
      $("f-gpus").onchange = (ev) => { form.gpus = { num: ev.target.value, vendor: form.gpus.vendor }; renderVendor(); };
      $("f-gpu-vendor").onchange = (ev) => {
        form.gpus = { num: form.gpus.num, vendor: ev.target.value };
        $("f-gpu-vendor-err").textContent = JWA.vendorError(form.gpus);
      };
      $("f-name").oninput = (ev) => {
        form.name = ev.target.value;
        if (form.workspace.enabled && form.workspace.type === "new") { form.workspace.name = JWA.volumeName(form.workspace.template, form.name); renderWorkspace(); }
      };
      $("f-type").onchange = (ev) => {
        form.serverType = ev.target.value;
        $("f-image-row").hidden = form.serverType !== "jupyter";
        $("f-image-g1-row").hidden = form.serverType !== "group-one";
        $("f-image-g2-row").hidden = form.serverType !== "group-two";
      };
      $("f-cpu").oninput = (ev) => { form.cpu = ev.target.value; if (!cpuLimitDirty) { form.cpuLimit = JWA.limitFrom(form.cpu, config.cpu.limitFactor, ""); $("f-cpu-limit").value = form.cpuLimit; } };
      $("f-mem").oninput = (ev) => { form.memory = ev.target.value; if (!memLimitDirty) { form.memoryLimit = JWA.limitFrom(form.memory, config.memory.limitFactor, "Gi"); $("f-mem-limit").value = form.memoryLimit; } };
      $("f-cpu-limit").oninput = (ev) => { cpuLimitDirty = true; form.cpuLimit = ev.target.value; };
      $("f-mem-limit").oninput = (ev) => { memLimitDirty = true; form.memoryLimit = ev.target.value; };
      $("f-ws").onchange = (ev) => { form.workspace.enabled = ev.target.checked; renderWorkspace(); };
      $("f-ws-kind").onchange = (ev) => { form.workspace = ev.target.value === "custom" ? JWA.toCustom(form.workspace) : JWA.fromCustom(form.workspace); renderWorkspace(); };
      $("f-ws-name").oninput = (ev) => { form.workspace.name = ev.target.value; form.workspace.template = ev.target.value; $("f-ws-header").textContent = ev.target.value; };
      $("f-ws-size").oninput = (ev) => { form.workspace.size = ev.target.value; };
      $("f-ws-sc-default").onchange = (ev) => { form.workspace.useDefaultSC = ev.target.checked; if (!ev.target.checked) form.workspace.storageClass = $("f-ws-sc").value; renderWorkspace(); };
      $("f-ws-sc").onchange = (ev) => { form.workspace.storageClass = ev.target.value; };
      document.querySelectorAll('input[name="f-ws-mode"]').forEach((r) => { r.onchange = () => { form.workspace.accessMode = r.value; }; });
      $("f-add-vol").onclick = () => { form.datavols.push(JWA.newDataVolume(form.name, form.datavols.length + 1)); renderDataVolumes(); };
    }

    async function openSpawner() {
      const ns = kf.namespace();
      form = JWA.formDefaults(config, "");
      cpuLimitDirty = memLimitDirty = false;
      $("f-name").value = "";
      try {
        const { poddefaults } = await kf.call("GET", `/api/namespaces/${ns}/poddefaults`);
        $("f-configs").innerHTML = poddefaults.map((pd) =>
          `<label class="muted"><input type="checkbox" value="${kf.esc(pd.label)}"${form.configurations.includes(pd.label) ? " checked" : ""}> ${kf.esc(pd.desc)}</label><br>`).join("") || '<span class="muted">none</span>';
      } catch (e) { $("f-configs").innerHTML = '<span class="muted">none</span>'; }
      try { form.pvcs = (await kf.call("GET", `/api/namespaces/${ns}/pvcs`)).pvcs; } catch (e) { form.pvcs = []; }
      // storage-class.component.ts: the cluster's classes and the default one
      try { form.storageClasses = (await kf.call("GET", "/api/storageclasses")).storageClasses; } catch (e) { form.storageClasses = []; }
      try { form.defaultStorageClass = (await kf.call("GET", "/api/storageclasses/default")).defaultStorageClass; } catch (e) { form.defaultStorageClass = ""; }
      // backend.service.ts getGPUVendors: the configured vendors some node reports capacity for
      try { installedVendors = new Set((await kf.call("GET", "/api/gpus")).vendors || []); } catch (e) { installedVendors = new Set(); }
      fillSpawner();
      $("f-error").textContent = "";
      $("spawner").showModal();
    }

    async function submit(ev) {
      if (ev.submitter && ev.submitter.value !== "ok") return;
      ev.preventDefault();
      const ns = kf.namespace();
      form.customImage = $("f-custom").value.trim();
      form.gpus = { num: $("f-gpus").value, vendor: $("f-gpu-vendor").value };
      $("f-gpu-vendor-err").textContent = JWA.vendorError(form.gpus);
      form.shm = $("f-shm").checked;
      form.affinityConfig = $("f-affinity").value || "none";
      form.tolerationGroup = $("f-toleration").value || "none";
      form.configurations = [...$("f-configs").querySelectorAll("input:checked")].map((i) => i.value);
      const errs = JWA.validate(form);
      if (errs.length) { $("f-error").textContent = errs.join("; "); return; }
      try {
        await kf.call("POST", `/api/namespaces/${ns}/notebooks`, JWA.buildBody(form, config, ns));
        $("spawner").close(); kf.snack(`Notebook ${form.name} created`, "SUCCESS"); poller.reset();
      } catch (e) { $("f-error").textContent = e.message; }
    }

    async function main() {
      poller = new kf.Poller(refresh);
      table = new kf.ResourceTable($("notebooks"), tableConfig());
      $("filter").oninput = (ev) => table.setFilter(ev.target.value);
      try {
        config = (await kf.call("GET", "/api/config")).config;
        await loadNamespaces();
      } catch (e) { kf.snack(e.message, "ERROR"); }
      form = JWA.formDefaults(config || {}, "");
      $("new").onclick = openSpawner;
      $("form").addEventListener("submit", submit);
      bindSpawner();
      kf.onNamespace((ns) => { if (!allNs) { $("ns").value = ns; poller.reset(); } });
      poller.start();
    }
    main();
  }

  global.JWA = JWA;
  if (typeof module !== "undefined" && module.exports) module.exports = JWA;  // node unit tests
  else if (typeof document !== "undefined") app();
})(typeof window !== "undefined" ? window : globalThis);
